set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05g}
SLIO_LIB=_var/libslio_STAMP.so timeout -k 10 300 python scripts/stamps_cert.py > gpurun_out/${tag}_stamps.log 2>&1 || { tail gpurun_out/${tag}_stamps.log; exit 7; }
cat gpurun_out/${tag}_stamps.log | grep cert
for n in 1 2 8; do timeout -k 10 300 python bench.py --workload group --group-ranks $n --steps 100 --warmup 10 > gpurun_out/${tag}_group$n.json 2>/dev/null || exit 6; done
python -c "
import json
for n in (1,2,8):
    d=json.load(open('gpurun_out/${tag}_group%d.json'%n)); print(n, round(d['value']), round(d['us_per_pass'],1), {k: round(v,1) for k,v in d['host_us_per_update'].items()})
"
