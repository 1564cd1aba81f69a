# round-3 session check: runtime/parity/map/chain GPU tests, in-process A/B of the
# block-row fit reload (FITB) and MFMA sums, C2 bench, live-mapping aux bench
timeout -k 10 500 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_parity.py tests/test_gpu_map.py tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03s7_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03s7_tests.log; grep -E "FAILED|Error" gpurun_out/r03s7_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/r03s7_mapping.jsonl 2>&1 || { echo "mapping failed"; tail gpurun_out/r03s7_mapping.jsonl; exit 6; }
cat gpurun_out/r03s7_mapping.jsonl
for k in 1 2; do
  timeout -k 10 300 python scripts/ab_inproc.py - SLIO_NO_MFMA=1 --rounds 5 | sed "s/^/main /" || exit 5
  SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_noFITB.so timeout -k 10 300 python scripts/ab_inproc.py - SLIO_NO_MFMA=1 --rounds 5 | sed "s/^/noFITB /" || exit 5
done > gpurun_out/r03s7_ab.log 2>&1
cat gpurun_out/r03s7_ab.log
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/r03s7_bench.json 2>gpurun_out/r03s7_bench.err; cat gpurun_out/r03s7_bench.json
