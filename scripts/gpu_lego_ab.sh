# one GPU call: the LeGO GPU tests, then bench.py --workload lego alternating
# an environment switch (off / on) and a rocprofv3 kernel trace of the default
# -> gpurun_out/<tag>_*
#   bash scripts/gpu_lego_ab.sh <tag> <VAR=value>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; sw=$2
timeout -k 10 600 python -u -m pytest tests/test_gpu_lego.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
for rep in 1 2 3; do
  for cfg in "$sw" "-"; do
    if [ "$cfg" = "-" ]; then envs=""; else envs="$cfg"; fi
    env $envs timeout -k 10 300 python bench.py --workload lego --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/${tag}_lego.json 2>gpurun_out/${tag}_lego.err || { tail -5 gpurun_out/${tag}_lego.err; exit 4; }
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_lego.json')); print('$cfg', round(d['value']), d['ms_per_step'])"
  done
done | tee gpurun_out/${tag}_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_lego -o run -- python bench.py --workload lego --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/${tag}_lego_prof.json 2>/dev/null || exit 5
