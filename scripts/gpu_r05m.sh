set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05m}
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runtime.py tests/test_gpu_comm.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 3; }
grep -E "passed|failed" gpurun_out/${tag}_tests.log | tail -3
timeout -k 10 300 python scripts/ab_inproc.py - SLIO_PERSIST=1 --rounds 5 > gpurun_out/${tag}_ab.log 2>&1 || { tail gpurun_out/${tag}_ab.log; exit 7; }
tail -2 gpurun_out/${tag}_ab.log
for k in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench$k.json 2>/dev/null || exit 6; done
python -c "
import json
for k in (1,2):
    d=json.load(open(f'gpurun_out/${tag}_bench{k}.json')); print(k, round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2), d['roofline']['launch_covers'])
"
