# A/B of the C2 search pass between library builds: bash scripts/ab_search.sh <tag> lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 python -c "from agi_lidar_slam_amd import synth; synth.make_problem(10_000_000, 100_000, pattern='avia', cache_dir='/tmp/slio_cache')" || exit 3
for rep in 1 2; do
  for lib in "$@"; do
    SLIO_LIB=$lib REPS=40 timeout -k 10 120 python scripts/run_search.py 2>/dev/null || { echo "ab $lib failed"; exit 3; }
  done
done | tee gpurun_out/${tag}_ab.log
