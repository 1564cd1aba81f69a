# PMC instruction / LDS counters of k_search_pass, tiled vs per-query search
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for t in 1 0; do
  SLIO_SEARCH_TILE=$t REPS=5 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex k_search_pass -d gpurun_out/pmct$t -o pmc --output-format csv -- python3 scripts/run_search.py > gpurun_out/pmct$t.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmct$t.log; exit 6; }
  python3 - "$t" <<'PY'
import csv, glob, sys
from collections import defaultdict
v = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmct{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("tile", sys.argv[1], {k: round(sum(x) / len(x)) for k, x in sorted(v.items())})
PY
done
