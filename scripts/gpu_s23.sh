# bisect: C5 50M single-replica replay, session-start tree (_old) vs current, same box
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s23}
for rep in 1 2; do
  for t in _old .; do
    ( cd $t && timeout -k 10 400 python scripts/bench_replay.py --replicas 1 --steps 30 --map-points 50000000 --cell 1.25 > /tmp/r.json 2>> /tmp/r.err ) || { echo "replay $t failed"; tail -5 /tmp/r.err; exit 4; }
    python3 -c "import json; d=json.load(open('/tmp/r.json')); print('$t', round(d['value']))" | tee -a gpurun_out/${tag}_bisect.log
  done
done
