# auto cell edge: GPU suite, smoke, C2 bench (auto edge) + rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s20}
bash scripts/gpu_round.sh ${tag} tests smoke || exit $?
grep -q " passed" gpurun_out/${tag}_tests.log && ! grep -q "failed" gpurun_out/${tag}_tests.log || { echo "tests not green"; exit 3; }
bash scripts/gpu_round.sh ${tag} bench prof
