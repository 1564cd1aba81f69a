set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05h}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lego.py > gpurun_out/${tag}_lego_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_lego_tests.log; exit 3; }
grep -E "passed|failed" gpurun_out/${tag}_lego_tests.log | tail -3
for cc in band; do
  if [ $cc = lds1 ]; then export SLIO_LEGO_CC_LDS1=1; else unset SLIO_LEGO_CC_LDS1; fi
  timeout -k 10 300 python bench.py --workload lego --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/${tag}_lego_$cc.json 2>gpurun_out/${tag}_lego_$cc.err || { tail gpurun_out/${tag}_lego_$cc.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/${tag}_lego_$cc.json')); print('$cc', round(d['value']), d['ms_per_step'])"
done
unset SLIO_LEGO_CC_LDS1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_lego_prof -o run -- python bench.py --workload lego --steps 100 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit 5
python - <<PY
import csv,glob
for f in glob.glob('gpurun_out/${tag}_lego_prof/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:50]:50s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.2f}")
PY
timeout -k 10 300 python bench.py --workload group --group-ranks 1 --steps 50 --warmup 5 > gpurun_out/${tag}_group1.json 2> gpurun_out/${tag}_group1.err || { tail -5 gpurun_out/${tag}_group1.err; exit 6; }
