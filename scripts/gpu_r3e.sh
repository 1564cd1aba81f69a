# round 3: IKF tests, bench x2, kernel-trace timeline
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r3e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runtime.py tests/test_capi.py tests/test_gpu_map.py tests/test_gpu_lio_s2m.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; grep -E "FAILED|Error" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_$v.json 2> gpurun_out/${tag}_bench.err || { echo bench failed; tail gpurun_out/${tag}_bench.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_$v.json'));print(round(d['value']), round(d['ms_per_step']*1e3,1), 'us/step search', round(d['roofline']['avg_launch_us'],1))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-kernel-timing > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 5; }
python scripts/timeline.py gpurun_out/${tag}_prof 320 > gpurun_out/${tag}_timeline.txt 2>&1 || { echo timeline failed; tail gpurun_out/${tag}_timeline.txt; exit 6; }
cat gpurun_out/${tag}_timeline.txt
