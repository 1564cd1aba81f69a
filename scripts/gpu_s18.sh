# 1.0 m default cell: GPU suite, smoke, C2 bench + rocprofv3, PMC traffic of the search pass
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s18}
bash scripts/gpu_round.sh ${tag} tests smoke || exit $?
grep -q " passed" gpurun_out/${tag}_tests.log && ! grep -q "failed" gpurun_out/${tag}_tests.log || { echo "tests not green"; exit 3; }
bash scripts/gpu_round.sh ${tag} bench prof || exit $?
bash scripts/pmc_search.sh ${tag}
