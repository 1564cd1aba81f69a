# PMC passes of every kernel of the C3 scan (LIO-SAM, scripts/run_lio.py: 6
# launches) and of the LeGO sweep (scripts/run_lego.py: 9 launches):
# FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md) ->
# gpurun_out/<tag>_{c3,lego}_traffic.json (per kernel, and summed per scan)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-pmcfe}
for W in c3 lego; do
  S=scripts/run_lio.py; [ $W = lego ] && S=scripts/run_lego.py
  K=k_lio_claim,k_lio_fill,k_lio_extract,k_fe_pick,k_fe_ring,k_lio_concat
  [ $W = lego ] && K=k_lego_claim,k_lego_fill,k_lego_ground,k_lego_cc_band,k_lego_rows,k_lego_deskew,k_fe_pick,k_fe_ring,k_lego_concat
  i=0
  for PMC in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    REPS=50 timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "k_lio_|k_lego_|k_fe_" -d gpurun_out/${tag}_${W}pmc$i -o pmc --output-format csv -- python3 $S > gpurun_out/${tag}_${W}pmc$i.log 2>&1 || { echo "pmc $W $i failed"; tail -3 gpurun_out/${tag}_${W}pmc$i.log; exit 6; }
  done
  PMC_KERNELS=$K PMC_WORKLOAD=$W python3 scripts/pmc_traffic.py gpurun_out/${tag}_${W}_traffic.json gpurun_out/${tag}_${W}pmc* || exit 7
done
