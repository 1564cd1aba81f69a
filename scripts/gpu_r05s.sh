set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05s}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python bench.py --workload c3 --steps 300 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit 6
f=$(find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${tag}_c3_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.reader(open('gpurun_out/${tag}_c3_kernel_stats.csv')))[1:]: print(r[0][:70], r[1], round(float(r[3])/1000,2))
"
