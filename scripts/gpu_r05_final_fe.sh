# C3 / LeGO bench lines against the committed feature-stage traffic profiles
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05h}
B="timeout -k 10 400 python bench.py"
$B --workload c3 > gpurun_out/${tag}_bench_c3.json 2>/dev/null || exit 5
$B --workload lego > gpurun_out/${tag}_bench_lego.json 2>/dev/null || exit 6
for n in c3 lego; do python -c "
import json; d=json.load(open('gpurun_out/${tag}_bench_$n.json')); rf=d['roofline']; print('$n', round(d['value']), rf['frac'], rf['traffic'])"; done
