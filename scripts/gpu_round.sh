# usage: bash scripts/gpu_round.sh <tag> <step>...   (one GPU box, steps chained, each under its own limit)
# steps: tests smoke bench benchc3 benchc5 prof profc3 timeline solve ustamps pmc
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
tag=$1; shift
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${tag}_tests.log; grep -E "FAILED|SKIPPED" gpurun_out/${tag}_tests.log | head
      [ $rc -eq 0 ] || exit $rc ;;
    t:*)
      # selected test files / node ids, comma-separated: t:tests/test_gpu_comm.py,tests/test_x.py::test_y
      sel=${step#t:}; sel=${sel//,/ }
      timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tsel.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${tag}_tsel.log; grep -E "FAILED|SKIPPED|Error" gpurun_out/${tag}_tsel.log | head
      [ $rc -eq 0 ] || exit $rc ;;
    benchref)
      timeout -k 10 600 python bench.py --steps 200 --warmup 5 --mode reference --iters 3 > gpurun_out/${tag}_benchref.json 2> gpurun_out/${tag}_benchref.err || { echo "benchref failed"; tail -20 gpurun_out/${tag}_benchref.err; exit 4; }
      cat gpurun_out/${tag}_benchref.json ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${tag}_smoke.log; exit 6; }
      tail -1 gpurun_out/${tag}_smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py --steps 200 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 4; }
      cat gpurun_out/${tag}_bench.json ;;
    benchc3)
      timeout -k 10 600 python bench.py --workload c3 --steps 500 --warmup 10 > gpurun_out/${tag}_benchc3.json 2> gpurun_out/${tag}_benchc3.err || { echo "benchc3 failed"; tail -20 gpurun_out/${tag}_benchc3.err; exit 4; }
      cat gpurun_out/${tag}_benchc3.json ;;
    benchlego)
      timeout -k 10 600 python bench.py --workload lego --steps 1000 --warmup 20 > gpurun_out/${tag}_benchlego.json 2> gpurun_out/${tag}_benchlego.err || { echo "benchlego failed"; tail -20 gpurun_out/${tag}_benchlego.err; exit 4; }
      cat gpurun_out/${tag}_benchlego.json ;;
    proflego)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_proflego -o run --output-format csv -- python3 bench.py --workload lego --steps 500 --warmup 10 --no-cpu-baseline > gpurun_out/${tag}_proflego.log 2>&1 || { echo "proflego failed"; tail -20 gpurun_out/${tag}_proflego.log; exit 5; }
      for f in $(find gpurun_out/${tag}_proflego -name "*kernel_stats.csv"); do head -20 $f | cut -c1-150; done ;;
    profref)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_profref -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --mode reference --iters 3 > gpurun_out/${tag}_profref.log 2>&1 || { echo "profref failed"; tail -20 gpurun_out/${tag}_profref.log; exit 5; }
      for f in $(find gpurun_out/${tag}_profref -name "*kernel_stats.csv"); do head -8 $f; done ;;
    ab)
      # same-box in-process A/B: this tree vs agi_lidar_slam_amd/_abl/libslio_prev.so, alternating
      for k in 1 2; do
        timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/main /" || exit 7
        SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_prev.so timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/prev /" || exit 7
      done > gpurun_out/${tag}_ab.log 2>&1
      cat gpurun_out/${tag}_ab.log ;;
    ab3)
      # same-box A/B: this tree (+ two-launch with / without chunk order) vs the previous commit's library
      # and the no-reuse-branch ablation
      for k in 1 2; do
        timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/main /" || exit 7
        SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_prev.so timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/prev /" || exit 7
        SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_noreuse.so timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/noreuse /" || exit 7
      done > gpurun_out/${tag}_ab3.log 2>&1
      cat gpurun_out/${tag}_ab3.log ;;
    abenv)
      # in-process A/B of environment switches of this library: ABENV="SLIO_X=1 SLIO_Y=1"
      timeout -k 10 400 python scripts/ab_inproc.py - $ABENV --rounds 7 > gpurun_out/${tag}_abenv.log 2>&1 || { tail gpurun_out/${tag}_abenv.log; exit 7; }
      cat gpurun_out/${tag}_abenv.log ;;
    tailenv)
      # tail stamps with and without the environment switch TAILENV (e.g. SLIO_NO_INTERLEAVE=1)
      SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_sstamp.so timeout -k 10 200 python scripts/tail_stamps.py > gpurun_out/${tag}_tail.log 2>&1 || exit 8
      env $TAILENV SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_sstamp.so timeout -k 10 200 python scripts/tail_stamps.py > gpurun_out/${tag}_tail_env.log 2>&1 || exit 8
      grep "per pass" gpurun_out/${tag}_tail.log gpurun_out/${tag}_tail_env.log ;;
    tail)
      SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_sstamp.so timeout -k 10 200 python scripts/tail_stamps.py > gpurun_out/${tag}_tail.log 2>&1 || { tail gpurun_out/${tag}_tail.log; exit 8; }
      grep maxit gpurun_out/${tag}_tail.log ;;
    chain)
      timeout -k 10 600 python scripts/bench_aux.py chain > gpurun_out/${tag}_chain.jsonl 2> gpurun_out/${tag}_chain.err || { echo "chain failed"; tail -20 gpurun_out/${tag}_chain.err; exit 9; }
      cut -c1-1500 gpurun_out/${tag}_chain.jsonl ;;
    profchain)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_profchain -o run --output-format csv -- python3 scripts/bench_aux.py chain > gpurun_out/${tag}_profchain.log 2>&1 || { echo "profchain failed"; tail -20 gpurun_out/${tag}_profchain.log; exit 5; }
      for f in $(find gpurun_out/${tag}_profchain -name "*kernel_stats.csv"); do head -30 $f | cut -c1-150; done ;;
    festamps)
      SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_fe.so timeout -k 10 200 python scripts/fe_stamps.py > gpurun_out/${tag}_festamps.log 2>&1 || { tail gpurun_out/${tag}_festamps.log; exit 8; }
      grep -v amdgpu.ids gpurun_out/${tag}_festamps.log ;;
    mapping)
      timeout -k 10 600 python scripts/bench_aux.py mapping > gpurun_out/${tag}_mapping.jsonl 2> gpurun_out/${tag}_mapping.err || { echo "mapping failed"; tail -20 gpurun_out/${tag}_mapping.err; exit 9; }
      cut -c1-1500 gpurun_out/${tag}_mapping.jsonl ;;
    benchc5)
      timeout -k 10 900 python bench.py --workload c5 --steps 50 --warmup 3 > gpurun_out/${tag}_benchc5.json 2> gpurun_out/${tag}_benchc5.err || { echo "benchc5 failed"; tail -20 gpurun_out/${tag}_benchc5.err; exit 4; }
      cat gpurun_out/${tag}_benchc5.json ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/${tag}_prof.log; exit 5; }
      for f in $(find gpurun_out/${tag}_prof -name "*kernel_stats.csv"); do head -8 $f; done ;;
    profc3)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_profc3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 300 --warmup 10 --no-cpu-baseline > gpurun_out/${tag}_profc3.log 2>&1 || { echo "profc3 failed"; tail -20 gpurun_out/${tag}_profc3.log; exit 5; }
      for f in $(find gpurun_out/${tag}_profc3 -name "*kernel_stats.csv"); do head -12 $f | cut -c1-150; done ;;
    timeline)
      timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_tl -o run --output-format csv -- python3 bench.py --steps 150 --warmup 3 --no-cpu-baseline --no-kernel-timing > gpurun_out/${tag}_tl.log 2>&1 || { echo "timeline failed"; tail -20 gpurun_out/${tag}_tl.log; exit 5; }
      python scripts/timeline.py gpurun_out/${tag}_tl 320 | tee gpurun_out/${tag}_timeline.txt ;;
    solve)
      SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_SOLVE.so timeout -k 10 200 python scripts/solve_stamps.py > gpurun_out/${tag}_solve.log 2>&1 || { echo "solve failed"; tail gpurun_out/${tag}_solve.log; exit 6; }
      grep -v amdgpu.ids gpurun_out/${tag}_solve.log ;;
    ustamps)
      timeout -k 10 200 python scripts/stamps_update.py > gpurun_out/${tag}_ustamps.log 2>&1 || { echo "ustamps failed"; tail gpurun_out/${tag}_ustamps.log; exit 5; }
      grep -v amdgpu.ids gpurun_out/${tag}_ustamps.log ;;
    pmc)
      bash scripts/pmc_search.sh ${tag} || exit $? ;;
    pmcfe)
      bash scripts/pmc_frontend.sh ${tag} || exit $?
      cat gpurun_out/${tag}_c3_traffic.json gpurun_out/${tag}_lego_traffic.json | cut -c1-400 ;;
  esac
done
