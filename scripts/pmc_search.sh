# PMC passes of k_search_pass on the C2 problem (voxel-ordered scan, the
# bench's step: 4 fused passes of the device-resident update): HBM traffic (FETCH_SIZE, WRITE_SIZE, separate passes per
# MI355X_MICROARCH.md), L2 hit/miss and instruction mix -> profiles/search_traffic.json
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-pmc}
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  MODE=update REPS=10 timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex k_search_pass -d gpurun_out/${tag}_pmc$i -o pmc --output-format csv -- python3 scripts/run_search.py > gpurun_out/${tag}_pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 gpurun_out/${tag}_pmc$i.log; exit 6; }
done
python3 scripts/pmc_traffic.py gpurun_out/${tag}_search_traffic.json gpurun_out/${tag}_pmc*
