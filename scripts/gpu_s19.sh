# C5 batched replay on the 50M map at the 1.0 m default cell
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s19}
for R in 1 16; do
  timeout -k 10 400 python scripts/bench_replay.py --replicas $R --steps 30 --map-points 50000000 >> gpurun_out/${tag}_replay.jsonl 2>> gpurun_out/${tag}_replay.err || { echo "replay $R failed"; tail -5 gpurun_out/${tag}_replay.err; exit 4; }
  tail -1 gpurun_out/${tag}_replay.jsonl | cut -c1-200
done
