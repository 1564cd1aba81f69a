# round 3: kernel-trace timeline of the C2 bench (gaps between launches, host gap between steps)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r3d}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-kernel-timing > gpurun_out/${tag}_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/${tag}_prof.log; exit 5; }
tail -2 gpurun_out/${tag}_prof.log
python scripts/timeline.py gpurun_out/${tag}_prof 320 > gpurun_out/${tag}_timeline.txt 2>&1 || { echo timeline failed; tail gpurun_out/${tag}_timeline.txt; exit 6; }
cat gpurun_out/${tag}_timeline.txt
