set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_runtime.py -k "fused" > gpurun_out/r05a_tests.log 2>&1 || { tail -30 gpurun_out/r05a_tests.log; exit 3; }
tail -2 gpurun_out/r05a_tests.log
timeout -k 10 300 python scripts/host_gap.py > gpurun_out/r05a_hostgap.json 2> gpurun_out/r05a_hostgap.err || { tail gpurun_out/r05a_hostgap.err; exit 4; }
for k in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05a_bench$k.json 2>/dev/null || exit 5; done
python -c "
import json
for k in (1,2):
    d=json.load(open(f'gpurun_out/r05a_bench{k}.json')); print(k, round(d['value']), round(d['ms_per_step']*1e3,1))
"
