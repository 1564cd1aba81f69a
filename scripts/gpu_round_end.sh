# round-end call A: full GPU suite + smoke, then bench part 1 (PMC traffic, C2 lines)
set -o pipefail
tag=${1:-r06e}
bash scripts/gpu_tests.sh $tag || exit $?
bash scripts/gpu_bench.sh $tag 1 || exit $?
