# A/B of bench.py between library builds on one box (scripts/variant.py, the
# in-tree library stays as built): bash scripts/ab_bench.sh <tag> <reps> lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; reps=$2; shift 2
for rep in $(seq $reps); do
  for lib in "$@"; do
    timeout -k 10 300 python scripts/variant.py $lib bench.py --steps 300 --warmup 10 --no-cpu-baseline 2>gpurun_out/${tag}_abbench.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))" || { echo "bench $lib failed"; tail -5 gpurun_out/${tag}_abbench.err; exit 4; }
  done
done | tee gpurun_out/${tag}_abbench.log
