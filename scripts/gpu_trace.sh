# usage: bash scripts/gpu_trace.sh <tag> [bench args...] — kernel + memcpy timeline of a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/${tag}_trace -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/${tag}_trace.log; exit 5; }
python3 scripts/timeline.py gpurun_out/${tag}_trace 240
