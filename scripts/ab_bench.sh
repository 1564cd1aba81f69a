# A/B of bench.py between library builds (copies each over the in-tree libslio.so
# of the box's scratch copy): bash scripts/ab_bench.sh <tag> lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    cp "$lib" agi_lidar_slam_amd/libslio.so || exit 3
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))" || { echo "bench $lib failed"; exit 4; }
  done
done | tee gpurun_out/${tag}_abbench.log
