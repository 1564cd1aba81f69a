set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r3l
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_parity.py tests/test_gpu_runtime.py tests/test_capi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; grep -E "FAILED|Error|SKIP" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh ${tag} 2 agi_lidar_slam_amd/_abl/libslio_B.so agi_lidar_slam_amd/_abl/libslio_F.so
