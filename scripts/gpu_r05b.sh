set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_runtime.py -k "certificate or fused or pinned" > gpurun_out/r05b_tests.log 2>&1 || { tail -40 gpurun_out/r05b_tests.log; exit 3; }
grep -E "passed|failed|certified" gpurun_out/r05b_tests.log | tail -12
for k in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05b_bench$k.json 2>/dev/null || exit 5; done
timeout -k 10 300 python scripts/ab_inproc.py - SLIO_NO_KNN_CERT=1 --rounds 5 > gpurun_out/r05b_ab.log 2>&1 || { tail gpurun_out/r05b_ab.log; exit 6; }
cat gpurun_out/r05b_ab.log | tail -4
python -c "
import json
for k in (1,2):
    d=json.load(open(f'gpurun_out/r05b_bench{k}.json')); print(k, round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))
"
