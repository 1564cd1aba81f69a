# one GPU call: the whole -m gpu suite, then C2 and LeGO bench lines
# (no CPU baselines) -> gpurun_out/<tag>_*
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 3; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 120 ./scripts/micro/launch_cost > gpurun_out/${tag}_launch_cost.jsonl 2>&1 || exit 6
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
$B --steps 200 --warmup 10 > gpurun_out/${tag}_bench_c2.json 2>gpurun_out/${tag}_bench_c2.err || exit 4
$B --workload lego > gpurun_out/${tag}_bench_lego.json 2>/dev/null || exit 5
timeout -k 10 300 python bench.py --workload s2m --steps 20 --warmup 2 > gpurun_out/${tag}_bench_s2m.json 2>gpurun_out/${tag}_bench_s2m.err || exit 7
python - <<PY
import json
for n in ("c2", "lego", "s2m"):
    d = json.load(open(f"gpurun_out/${tag}_bench_{n}.json"))
    print(n, round(d["value"]), round(d["ms_per_step"] * 1e3, 1), d["roofline"]["avg_launch_us"])
PY
