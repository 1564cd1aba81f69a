set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05s}
for w in c3 lego; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_$w -o run -- python bench.py --workload $w --steps 300 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit 6
f=$(find gpurun_out/${tag}_prof_$w -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${tag}_${w}_kernel_stats.csv
python3 -c "
import csv
for r in list(csv.reader(open('gpurun_out/${tag}_${w}_kernel_stats.csv')))[1:]: print(r[0][:60], r[1], round(float(r[3])/1000,2))
"
done
