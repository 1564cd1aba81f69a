# round-3 session: same-box A/B of the block-row fit reload (previous commit's
# build in _abl), live-mapping aux bench merge vs sort, rocprof of the live path
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/main /" || exit 5
  SLIO_LIB_OVERRIDE=agi_lidar_slam_amd/_abl/libslio_fitb.so timeout -k 10 300 python scripts/ab_inproc.py - --rounds 5 | sed "s/^/fitb /" || exit 5
done > gpurun_out/r03s8_ab.log 2>&1
cat gpurun_out/r03s8_ab.log
timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/r03s8_mapping.jsonl 2>&1 || { echo "mapping failed"; tail gpurun_out/r03s8_mapping.jsonl; exit 6; }
SLIO_NO_MERGE=1 timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/r03s8_mapping_sort.jsonl 2>&1 || { echo "mapping sort failed"; exit 6; }
cat gpurun_out/r03s8_mapping.jsonl gpurun_out/r03s8_mapping_sort.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03s8_mprof -o run --output-format csv -- python3 scripts/bench_aux.py mapping > gpurun_out/r03s8_mprof.log 2>&1 || { echo "mapping prof failed"; tail gpurun_out/r03s8_mprof.log; exit 7; }
echo prof ok
