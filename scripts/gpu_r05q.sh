set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05q}
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runtime.py tests/test_gpu_parity.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 3; }
grep -E "passed|failed" gpurun_out/${tag}_tests.log | tail -3
bash scripts/ab_bench.sh $tag 3 agi_lidar_slam_amd/libslio.so _var/libslio_head.so || exit 3
