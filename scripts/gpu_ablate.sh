set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
python -c "from agi_lidar_slam_amd import synth; synth.make_problem(10_000_000, 100_000, pattern='avia', cache_dir='/tmp/slio_cache')"
for V in FULL NOFIT NOCAND IO; do
  for C in 1.0 1.25; do
    SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_$V.so LPQ=2 CELL=$C timeout -k 10 120 python scripts/run_search.py 2>/dev/null || { echo "abl $V failed"; exit 3; }
  done
done | tee gpurun_out/${tag}_ablate.log
# PMC passes on the full library (LPQ 2, cell 1.0), one counter group per pass
i=0
for PMC in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  LPQ=2 CELL=1.0 REPS=5 timeout -k 10 180 rocprofv3 --pmc $PMC --kernel-include-regex k_search_pass -d gpurun_out/${tag}_pmc$i -o pmc --output-format csv -- python3 scripts/run_search.py > gpurun_out/${tag}_pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/${tag}_pmc$i.log; }
done
for f in $(find gpurun_out/${tag}_pmc* -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if "search" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, "n=%d" % len(v), "mean=%.4g" % (sum(v) / len(v)))
PY
done
