# usage: bash scripts/gpu_round.sh <tag> [tests] [sweep] [bench] [prof]
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1; shift
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/${tag}_tests.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    fetests)
      timeout -k 10 600 python -m pytest tests/test_gpu_frontend.py tests/test_gpu_lego.py -m gpu -q -rs > gpurun_out/${tag}_fetests.log 2>&1
      rc=$?; echo "fetests rc=$rc"; tail -40 gpurun_out/${tag}_fetests.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${tag}_smoke.log; exit 6; }
      tail -3 gpurun_out/${tag}_smoke.log ;;
    sweep)
      timeout -k 10 600 python scripts/sweep_search.py > gpurun_out/${tag}_sweep.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/${tag}_sweep.log; exit 3; }
      cat gpurun_out/${tag}_sweep.log | grep -v amdgpu.ids ;;
    bench)
      timeout -k 10 600 python bench.py --steps 100 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 4; }
      cat gpurun_out/${tag}_bench.json ;;
    benchc3)
      timeout -k 10 600 python bench.py --workload c3 --steps 500 --warmup 10 > gpurun_out/${tag}_benchc3.json 2> gpurun_out/${tag}_benchc3.err || { echo "benchc3 failed"; tail -20 gpurun_out/${tag}_benchc3.err; exit 4; }
      cat gpurun_out/${tag}_benchc3.json ;;
    benchh)
      timeout -k 10 600 python bench.py --steps 100 --warmup 5 --host-loop --no-cpu-baseline > gpurun_out/${tag}_benchh.json 2> gpurun_out/${tag}_benchh.err || { echo "benchh failed"; tail -20 gpurun_out/${tag}_benchh.err; exit 4; }
      cat gpurun_out/${tag}_benchh.json ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/${tag}_prof.log; exit 5; }
      find gpurun_out/${tag}_prof -name "*stats*" | head; for f in $(find gpurun_out/${tag}_prof -name "*kernel_stats.csv"); do head -8 $f; done ;;
  esac
done
