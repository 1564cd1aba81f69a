# search pass time vs grid cell edge (C2, voxel order): bash scripts/cell_sweep.sh <tag> cells...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 python -c "from agi_lidar_slam_amd import synth; synth.make_problem(10_000_000, 100_000, pattern='avia', cache_dir='/tmp/slio_cache')" || exit 3
for c in "$@"; do
  CELL=$c REPS=40 timeout -k 10 120 python scripts/run_search.py 2>/dev/null || { echo "cell $c failed"; exit 3; }
done | tee gpurun_out/${tag}_cells.log
