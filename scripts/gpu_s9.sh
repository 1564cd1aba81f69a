# round-3 session: map/chain/runtime GPU tests after the rebuild changes, live-mapping aux bench + rocprof
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_chain.py tests/test_gpu_far.py tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03s11_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03s11_tests.log; grep -E "FAILED|Error" gpurun_out/r03s11_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/r03s11_mapping.jsonl 2>&1 || { echo "mapping failed"; tail gpurun_out/r03s11_mapping.jsonl; exit 6; }
cat gpurun_out/r03s11_mapping.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03s11_mprof -o run --output-format csv -- python3 scripts/bench_aux.py mapping > gpurun_out/r03s11_mprof.log 2>&1 || { echo "mapping prof failed"; tail gpurun_out/r03s11_mprof.log; exit 7; }
echo prof ok
