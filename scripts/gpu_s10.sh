# live-mapping rebuilds: which take the cell-only sort (SLIO_DEBUG_REBUILD)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s10}
SLIO_DEBUG_REBUILD=1 timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/${tag}_aux.jsonl 2> gpurun_out/${tag}_aux.err || { tail -5 gpurun_out/${tag}_aux.err; exit 4; }
cat gpurun_out/${tag}_aux.jsonl; grep "slio rebuild" gpurun_out/${tag}_aux.err | head -20
