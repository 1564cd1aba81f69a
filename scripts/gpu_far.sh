# usage: bash scripts/gpu_far.sh <tag>   (far-path tests, full GPU suite, bench)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_far.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_far.log 2>&1
rc=$?; echo "far rc=$rc"; tail -15 gpurun_out/${tag}_far.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.err; exit 4; }
cat gpurun_out/${tag}_bench.json
