# one GPU call: the front-end GPU tests, PMC traffic of every front-end kernel
# (C3 and LeGO), the C3 / LeGO bench lines and their kernel statistics
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_lego.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
bash scripts/pmc_frontend.sh $tag || exit 4
B="timeout -k 10 300 python bench.py"
$B --workload c3 > gpurun_out/${tag}_bench_c3.json 2>gpurun_out/${tag}_bench_c3.err || exit 5
$B --workload lego > gpurun_out/${tag}_bench_lego.json 2>gpurun_out/${tag}_bench_lego.err || exit 6
for w in c3 lego; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_$w -o run -- python bench.py --workload $w --steps 100 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit 7
  f=$(find gpurun_out/${tag}_prof_$w -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${tag}_${w}_kernel_stats.csv
done
python3 - <<PY
import json
for n in ("c3", "lego"):
    d = json.load(open(f"gpurun_out/${tag}_bench_{n}.json"))
    r, f = d["roofline"], d["roofline_feature_stage"]
    print(n, round(d["value"]), round(d["ms_per_step"] * 1e3, 1), "scan", round(r["avg_launch_us"], 1), r["frac"], r["traffic"], "feat", round(f["avg_launch_us"], 1), f["traffic"])
PY
