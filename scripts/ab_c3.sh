# same-box A/B of the C3 front-end between library builds: bash scripts/ab_c3.sh <tag> <reps> <streams> lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; reps=$2; S=$3; shift 3
for rep in $(seq $reps); do
  for lib in "$@"; do
    timeout -k 10 300 python scripts/variant.py $lib bench.py --workload c3 --steps 500 --warmup 10 --c3-streams $S --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib S=$S', round(d['value']), round(d['roofline']['avg_launch_us'],2))" || { echo "bench $lib failed"; exit 4; }
  done
done | tee -a gpurun_out/${tag}_abc3.log
