set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05j}
SLIO_LIB=_var/libslio_fe.so timeout -k 10 120 python scripts/band_stamps.py > gpurun_out/${tag}_band.log 2>&1 || { tail gpurun_out/${tag}_band.log; exit 2; }
cat gpurun_out/${tag}_band.log | grep band
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runtime.py -k "certificate or fused or pinned or reference_gain" > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 3; }
grep -E "passed|failed|certified" gpurun_out/${tag}_tests.log | tail -12
timeout -k 10 300 python scripts/cert_probe.py > gpurun_out/${tag}_probe.log 2>&1 || { tail gpurun_out/${tag}_probe.log; exit 4; }
cat gpurun_out/${tag}_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_prof -o run -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline --timing-steps 1 > gpurun_out/${tag}_b1.json 2>/dev/null || exit 5
python scripts/pass_times.py gpurun_out/${tag}_prof 4 40
for k in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench$k.json 2>/dev/null || exit 6; done
timeout -k 10 300 python scripts/ab_inproc.py - SLIO_NO_KNN_CERT=1 --rounds 5 > gpurun_out/${tag}_ab.log 2>&1 || { tail gpurun_out/${tag}_ab.log; exit 7; }
tail -2 gpurun_out/${tag}_ab.log
python -c "
import json
for k in (1,2):
    d=json.load(open(f'gpurun_out/${tag}_bench{k}.json')); print(k, round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))
"
