# usage: bash scripts/lio_kstats.sh <tag> [SLIO_LIB] -- per-kernel averages of the C3 front-end
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; lib=${2:-}
if [ -n "$lib" ]; then export SLIO_LIB=$lib; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag} -o run --output-format csv -- python3 scripts/run_lio.py > gpurun_out/${tag}.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${tag}.log; exit 5; }
grep scans gpurun_out/${tag}.log
python3 - gpurun_out/${tag}/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:40]:42s} calls {r["Calls"]:>5} avg {float(r["AverageNs"])/1e3:8.2f} us')
PY
