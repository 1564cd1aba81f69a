set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05r}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frontend.py tests/test_gpu_lego.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 3; }
grep -E "passed|failed" gpurun_out/${tag}_tests.log | tail -3
bash scripts/ab_c3.sh $tag 2 1 agi_lidar_slam_amd/libslio.so _var/libslio_head.so || exit 4
for lib in agi_lidar_slam_amd/libslio.so _var/libslio_head.so agi_lidar_slam_amd/libslio.so _var/libslio_head.so; do
  timeout -k 10 300 python scripts/variant.py $lib bench.py --workload lego --steps 500 --warmup 10 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib lego', round(d['value']))" || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python bench.py --workload c3 --steps 300 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit 6
find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${tag}_c3_kernel_stats.csv
