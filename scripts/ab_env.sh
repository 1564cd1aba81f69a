# A/B of bench.py between environment settings on one box (same library):
# bash scripts/ab_env.sh <tag> <reps> "ENV=1 ..." "ENV=0" ...   ("-" = no extra env)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; reps=$2; shift 2
for rep in $(seq $reps); do
  for e in "$@"; do
    ee="$e"; [ "$ee" = "-" ] && ee=""
    env $ee timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))" || { echo "bench $e failed"; exit 4; }
  done
done | tee gpurun_out/${tag}_abenv.log
