set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
python -c "from agi_lidar_slam_amd import synth; synth.make_problem(10_000_000, 100_000, pattern='avia', cache_dir='/tmp/slio_cache')"
{
for cfg in "2 1.25 0" "2 1.0 0" "2 1.5 0" "1 1.25 0" "4 1.25 0" "2 0.75 1.0" "2 1.0 1.2"; do
  set -- $cfg
  LPQ=$1 CELL=$2 RADIUS=$3 timeout -k 10 120 python scripts/run_search.py 2>/dev/null || exit 3
done
for N in 25000 50000; do LPQ=2 CELL=1.25 RADIUS=0 NSCAN=$N timeout -k 10 120 python scripts/run_search.py 2>/dev/null || exit 3; done
} | tee gpurun_out/${tag}_exp.log
