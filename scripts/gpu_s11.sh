# rebuild keeps its grid: map tests, live-mapping timing per rebuild, rocprof of the live loop
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s11}
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_runtime.py tests/test_gpu_far.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_maptests.log 2>&1; rc=$?
tail -4 gpurun_out/${tag}_maptests.log; [ $rc -eq 0 ] || exit 3
SLIO_DEBUG_REBUILD=1 timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/${tag}_aux.jsonl 2> gpurun_out/${tag}_aux.err || { tail -5 gpurun_out/${tag}_aux.err; exit 4; }
cat gpurun_out/${tag}_aux.jsonl; grep "slio rebuild" gpurun_out/${tag}_aux.err | cut -c1-60
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 scripts/bench_aux.py mapping > gpurun_out/${tag}_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${tag}_prof.log; exit 5; }
