export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_chain.py tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03i_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03i_tests.log; grep -E "FAILED|Error" gpurun_out/r03i_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/r03i_mapping.jsonl 2>&1 || { echo "mapping failed"; tail gpurun_out/r03i_mapping.jsonl; exit 6; }
cut -c1-400 gpurun_out/r03i_mapping.jsonl
timeout -k 10 400 python scripts/ab_inproc.py - SLIO_EVENT_WAIT=1 --rounds 7 > gpurun_out/r03i_ab.log 2>&1 || { echo "ab failed"; tail gpurun_out/r03i_ab.log; exit 5; }
cat gpurun_out/r03i_ab.log
