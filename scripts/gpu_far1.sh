# usage: bash scripts/gpu_far1.sh <tag> <pytest -k expr>
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 150 python -u -m pytest tests/test_gpu_far.py -m gpu -x -v -s --timeout 100 --timeout-method thread -k "$2" > gpurun_out/${tag}_far.log 2>&1
rc=$?; echo "far rc=$rc"; tail -30 gpurun_out/${tag}_far.log
exit $rc
