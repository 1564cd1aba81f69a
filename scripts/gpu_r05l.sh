set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05l}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_comm.py > gpurun_out/${tag}_comm.log 2>&1 || { tail -40 gpurun_out/${tag}_comm.log; exit 3; }
grep -E "passed|failed" gpurun_out/${tag}_comm.log | tail -3
for n in 2 4 8; do timeout -k 10 300 python bench.py --workload group --group-ranks $n --steps 100 --warmup 10 > gpurun_out/${tag}_group$n.json 2>gpurun_out/${tag}_group$n.err || { tail -5 gpurun_out/${tag}_group$n.err; exit 4; }; done
for n in 2 8; do SLIO_NO_FUSE=1 timeout -k 10 300 python bench.py --workload group --group-ranks $n --steps 100 --warmup 10 > gpurun_out/${tag}_group${n}_nofuse.json 2>/dev/null || exit 5; done
python -c "
import json
for n in ('2','4','8','2_nofuse','8_nofuse'):
    d=json.load(open('gpurun_out/${tag}_group%s.json'%n)); print(n, round(d['value']), round(d['us_per_pass'],1), {k: round(v,1) for k,v in d['host_us_per_update'].items()})
"
