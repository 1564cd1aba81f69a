# one GPU call: the map / chain GPU tests, then the live chain against a
# variant build (_var/libslio_base.so, scripts/build_variant.sh) and under
# rocprofv3 -> gpurun_out/<tag>_*
#   bash scripts/gpu_chain_ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-chain_ab}
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_chain.py tests/test_gpu_lio_s2m.py tests/test_gpu_imu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
for rep in 1 2; do
  timeout -k 10 300 python scripts/variant.py _var/libslio_base.so scripts/bench_aux.py chain > gpurun_out/${tag}_chain_base$rep.jsonl 2>/dev/null || exit 4
  timeout -k 10 300 python scripts/bench_aux.py chain > gpurun_out/${tag}_chain_new$rep.jsonl 2>/dev/null || exit 5
done
python3 - "$tag" <<'PY'
import json, sys
tag = sys.argv[1]
for t in ("base1", "new1", "base2", "new2"):
    for line in open(f"gpurun_out/{tag}_chain_{t}.jsonl"):
        d = json.loads(line)
        if d.get("bench") == "live_chain_per_scan":
            print(t, round(d["ms_per_scan_mapping"], 3), {k: round(v, 3) for k, v in d["median"].items()})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_chain -o run -- python scripts/bench_aux.py chain > gpurun_out/${tag}_chain_prof.jsonl 2>/dev/null || exit 6
