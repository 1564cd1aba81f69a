# usage: bash scripts/gpu_step.sh <tag> [far] [tests] [stats "N S ..."] [bench]
# runs the named steps in order, each under its own time limit; stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
while [ $# -gt 0 ]; do
  case $1 in
    far) timeout -k 10 300 python -u -m pytest tests/test_gpu_far.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_far.log 2>&1
         rc=$?; echo "far rc=$rc"; tail -4 gpurun_out/${tag}_far.log; [ $rc -eq 0 ] || exit $rc ;;
    runtime) timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_runtime.log 2>&1
         rc=$?; echo "runtime rc=$rc"; tail -15 gpurun_out/${tag}_runtime.log; [ $rc -eq 0 ] || exit $rc ;;
    map) timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_map.log 2>&1
         rc=$?; echo "map rc=$rc"; tail -25 gpurun_out/${tag}_map.log; [ $rc -eq 0 ] || exit $rc ;;
    imu) timeout -k 10 300 python -u -m pytest tests/test_gpu_imu.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${tag}_imu.log 2>&1
         rc=$?; echo "imu rc=$rc"; tail -25 gpurun_out/${tag}_imu.log; [ $rc -eq 0 ] || exit $rc ;;
    s2m) timeout -k 10 300 python -u -m pytest tests/test_gpu_lio_s2m.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/${tag}_s2m.log 2>&1
         rc=$?; echo "s2m rc=$rc"; tail -25 gpurun_out/${tag}_s2m.log; [ $rc -eq 0 ] || exit $rc ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
         rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    stats) shift; timeout -k 10 600 python -u scripts/far_stats.py $1 > gpurun_out/${tag}_stats.log 2>&1
         rc=$?; echo "stats rc=$rc"; cat gpurun_out/${tag}_stats.log | grep '^{'; [ $rc -eq 0 ] || exit $rc ;;
    bench) timeout -k 10 600 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
         rc=$?; echo "bench rc=$rc"; cat gpurun_out/${tag}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${tag}_bench.err; exit $rc; } ;;
    stamps) LPQS=2 timeout -k 10 300 python -u scripts/stamps.py > gpurun_out/${tag}_stamps.log 2>&1
         rc=$?; echo "stamps rc=$rc"; cat gpurun_out/${tag}_stamps.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $1"; exit 9 ;;
  esac
  shift
done
