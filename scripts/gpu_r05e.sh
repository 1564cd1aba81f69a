set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05e}
SLIO_NO_KNN_CERT=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_prof_cert -o run -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline --timing-steps 1 > gpurun_out/${tag}_b1.json 2>/dev/null || exit 4
python scripts/pass_times.py gpurun_out/${tag}_prof_cert 4 40
timeout -k 10 300 python scripts/cert_probe.py > gpurun_out/${tag}_probe.log 2>&1 || { tail gpurun_out/${tag}_probe.log; exit 3; }
cat gpurun_out/${tag}_probe.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runtime.py -k "certificate or reference_gain" > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 5; }
grep -E "passed|failed|certified|differing" gpurun_out/${tag}_tests.log | tail -20
for n in 1 2 8; do timeout -k 10 300 python bench.py --workload group --group-ranks $n --steps 100 --warmup 10 > gpurun_out/${tag}_group$n.json 2>/dev/null || exit 6; done
python -c "
import json
for n in (1,2,8):
    d=json.load(open('gpurun_out/${tag}_group%d.json'%n)); print(n, round(d['value']), round(d['us_per_pass'],1), d['host_us_per_update'])
"
SLIO_LIB=_var/libslio_STAMP.so timeout -k 10 300 python scripts/stamps_cert.py > gpurun_out/${tag}_stamps.log 2>&1 || { tail gpurun_out/${tag}_stamps.log; exit 7; }
cat gpurun_out/${tag}_stamps.log | grep cert
