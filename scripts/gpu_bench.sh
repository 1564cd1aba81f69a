# round-end measurements: PMC traffic for the final sources (C2 search pass;
# every C3 / LeGO front-end kernel), then the bench lines, kernel statistics,
# the C2 pass timeline, the live chain and the scan-to-map line
# -> gpurun_out/<tag>_*   (part 1: PMC + C2; part 2: the other workloads)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06b}
part=${2:-1}
B="timeout -k 10 400 python bench.py"
if [ $part = 1 ]; then
bash scripts/pmc_search.sh $tag || exit 2
bash scripts/pmc_frontend.sh $tag || exit 3
cp gpurun_out/${tag}_search_traffic.json profiles/search_traffic.json
cp gpurun_out/${tag}_c3_traffic.json profiles/c3_traffic.json
cp gpurun_out/${tag}_lego_traffic.json profiles/lego_traffic.json
$B > gpurun_out/${tag}_bench_c2.json 2>gpurun_out/${tag}_bench_c2.err || exit 4
$B --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench_c2_driver_setting.json 2>/dev/null || exit 4
$B --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/${tag}_bench_c2_200steps.json 2>/dev/null || exit 4
$B --mode reference --iters 3 > gpurun_out/${tag}_bench_c2_reference.json 2>/dev/null || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_c2 -o run -- python bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline --no-python-reference > /dev/null 2>&1 || exit 9
f=$(find gpurun_out/${tag}_prof_c2 -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${tag}_c2_kernel_stats.csv
python scripts/pass_times.py gpurun_out/${tag}_prof_c2 4 40 > gpurun_out/${tag}_c2_pass_times.txt
python scripts/timeline.py gpurun_out/${tag}_prof_c2 > gpurun_out/${tag}_c2_timeline.txt 2>&1 || true
cat gpurun_out/${tag}_c2_pass_times.txt
for n in c2 c2_driver_setting c2_200steps c2_reference; do python -c "
import json; d=json.load(open('gpurun_out/${tag}_bench_'+'$n'+'.json')); rf=d['roofline']; print('$n', round(d['value']), round(d['ms_per_step']*1e3,1), rf['frac'], rf['traffic'], d['config'].get('python_loop_value'))"; done
exit 0
fi
$B --workload c3 > gpurun_out/${tag}_bench_c3.json 2>/dev/null || exit 5
for S in 2 4; do $B --workload c3 --c3-streams $S --no-cpu-baseline > gpurun_out/${tag}_bench_c3_streams$S.json 2>/dev/null || exit 5; done
$B --workload lego > gpurun_out/${tag}_bench_lego.json 2>/dev/null || exit 6
$B --workload c5 --no-cpu-baseline > gpurun_out/${tag}_bench_c5.json 2>/dev/null || exit 7
for N in 2 8; do $B --workload group --group-ranks $N --steps 100 --warmup 10 > gpurun_out/${tag}_bench_group$N.json 2>/dev/null || exit 8; done
$B --workload s2m > gpurun_out/${tag}_bench_s2m.json 2>/dev/null || exit 10
for w in c3 lego s2m; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_$w -o run -- python bench.py --workload $w --steps 100 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit 9
  f=$(find gpurun_out/${tag}_prof_$w -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${tag}_${w}_kernel_stats.csv
done
timeout -k 10 300 python scripts/bench_aux.py chain > gpurun_out/${tag}_live_chain.jsonl 2>gpurun_out/${tag}_live_chain.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_chain -o run -- python scripts/bench_aux.py chain > /dev/null 2>&1 || exit 12
f=$(find gpurun_out/${tag}_prof_chain -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${tag}_chain_kernel_stats.csv
python - <<PY
import json
for n in ("c3", "c3_streams2", "c3_streams4", "lego", "c5", "group2", "group8", "s2m"):
    d = json.load(open(f"gpurun_out/${tag}_bench_{n}.json"))
    rf = d.get("roofline") or {}
    print(n, round(d["value"]), d["unit"], round(d.get("ms_per_step", 0) * 1e3, 1), "frac", rf.get("frac"), "traffic", rf.get("traffic"))
for line in open("gpurun_out/${tag}_live_chain.jsonl"):
    d = json.loads(line)
    if d.get("bench") == "live_chain_per_scan":
        print("chain", round(d["ms_per_scan_mapping"], 3), {k: round(v, 3) for k, v in d["median"].items()})
PY
