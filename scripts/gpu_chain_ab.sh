set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_chain.py tests/test_gpu_lio_s2m.py tests/test_gpu_imu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g_tests.log 2>&1 || { tail -30 gpurun_out/r06g_tests.log; exit 3; }
tail -1 gpurun_out/r06g_tests.log
for rep in 1 2; do
  timeout -k 10 300 python scripts/variant.py _var/libslio_base.so scripts/bench_aux.py chain > gpurun_out/r06g_chain_base$rep.jsonl 2>/dev/null || exit 4
  timeout -k 10 300 python scripts/bench_aux.py chain > gpurun_out/r06g_chain_new$rep.jsonl 2>/dev/null || exit 5
done
python3 - <<'PY'
import json
for t in ("base1", "new1", "base2", "new2"):
    for line in open(f"gpurun_out/r06g_chain_{t}.jsonl"):
        d = json.loads(line)
        if d.get("bench") == "live_chain_per_scan":
            print(t, round(d["ms_per_scan_mapping"], 3), {k: round(v, 3) for k, v in d["median"].items()})
PY
timeout -k 10 300 python bench.py --workload s2m --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r06g_bench_s2m.json 2>/dev/null && python3 -c "import json; d=json.load(open('gpurun_out/r06g_bench_s2m.json')); print('s2m', round(d['value']), d['ms_per_step'])"
