# bench + kernel-trace stats + PMC traffic for the committed profiles/
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
timeout -k 10 600 python bench.py --steps 30 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo "bench failed"; tail gpurun_out/${tag}_bench.err; exit 4; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || { echo "prof failed"; tail gpurun_out/${tag}_prof.log; exit 5; }
head -4 gpurun_out/${tag}_prof/run_kernel_stats.csv | cut -c1-220
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  REPS=10 timeout -k 10 180 rocprofv3 --pmc $PMC --kernel-include-regex k_search_pass -d gpurun_out/${tag}_pmc$i -o pmc --output-format csv -- python3 scripts/run_search.py > gpurun_out/${tag}_pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 gpurun_out/${tag}_pmc$i.log; exit 6; }
done
python scripts/pmc_traffic.py gpurun_out/${tag}_traffic.json gpurun_out/${tag}_pmc*
