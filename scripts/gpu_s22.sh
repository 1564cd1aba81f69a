# C5 50M replay: explicit 1.25 m vs auto edge, same box
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s22}
for cell in 1.25 0; do
  for R in 1 16; do
    timeout -k 10 400 python scripts/bench_replay.py --replicas $R --steps 30 --map-points 50000000 --cell $cell > gpurun_out/${tag}_r.json 2>> gpurun_out/${tag}_replay.err || { echo "replay failed"; tail -5 gpurun_out/${tag}_replay.err; exit 4; }
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_r.json')); print('cell $cell R $R', round(d['value']))" | tee -a gpurun_out/${tag}_replay.log
  done
done
