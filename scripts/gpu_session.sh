# round-3 session check: fused-pass GPU tests, tail stamps, same-box in-process A/B vs the previous tree
export TMPDIR=/tmp
tag=${1:-r03n}
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${tag}_tests.log 2>&1 || { tail -20 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_sstamp.so timeout -k 10 200 python scripts/tail_stamps.py > gpurun_out/${tag}_tail.log 2>&1 || { tail gpurun_out/${tag}_tail.log; exit 4; }
grep maxit gpurun_out/${tag}_tail.log
for k in 1 2; do
  timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/main /" || exit 5
  SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_prev.so timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/prev /" || exit 5
done > gpurun_out/${tag}_ab.log 2>&1
cat gpurun_out/${tag}_ab.log
