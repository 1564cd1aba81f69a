set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=r3k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-kernel-timing > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 5; }
python scripts/timeline.py gpurun_out/${tag}_prof 240
SLIO_NO_CHUNK_ORDER=1 timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no-order', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))"
SLIO_NO_FUSE=1 timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no-fuse', round(d['value']), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],2))"
