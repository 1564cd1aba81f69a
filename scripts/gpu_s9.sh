# map rebuild with the cell-only key: map GPU tests, the live-mapping timing
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s9}
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_runtime.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_maptests.log 2>&1; rc=$?
tail -4 gpurun_out/${tag}_maptests.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/${tag}_aux.jsonl 2> gpurun_out/${tag}_aux.err || { tail -5 gpurun_out/${tag}_aux.err; exit 4; }
cat gpurun_out/${tag}_aux.jsonl
