# session-6 GPU call: A/B of the lazy neighbour outputs, the full GPU suite,
# a 2-rank gloo rehearsal of bench.py's multi-rank path on one GPU, bench,
# rocprofv3 stats and the search pass's PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s6}
true
cp agi_lidar_slam_amd/_abl/libslio_lazy.so agi_lidar_slam_amd/libslio.so || exit 3
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo > gpurun_out/${tag}_gloo2.json 2> gpurun_out/${tag}_gloo2.err || { echo "gloo2 failed"; tail -20 gpurun_out/${tag}_gloo2.err; exit 4; }
cat gpurun_out/${tag}_gloo2.json
bash scripts/gpu_round.sh ${tag} tests smoke bench prof || exit $?
bash scripts/pmc_search.sh ${tag}
LPQS=2 timeout -k 10 180 python scripts/stamps.py > gpurun_out/${tag}_stamps.log 2>&1; tail -30 gpurun_out/${tag}_stamps.log
