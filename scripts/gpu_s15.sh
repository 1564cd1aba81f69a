# grid cell edge sweep of the C2 bench on the street scene
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s15}
for rep in 1 2; do
  for cell in 0.9 0.85 0.8 0.75 0.7; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --cell $cell 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cell', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))" || { echo "bench $cell failed"; exit 4; }
  done
done | tee gpurun_out/${tag}_cells.log
