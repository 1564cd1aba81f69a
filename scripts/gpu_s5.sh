# session-5 GPU call: store-coalescing A/B, then the full GPU suite, bench and
# rocprofv3 stats of the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s5}
bash scripts/ab_bench.sh ${tag} agi_lidar_slam_amd/_abl/libslio_base.so agi_lidar_slam_amd/_abl/libslio_coal.so agi_lidar_slam_amd/_abl/libslio_nostore.so || exit 3
cp agi_lidar_slam_amd/_abl/libslio_coal.so agi_lidar_slam_amd/libslio.so || exit 3
bash scripts/gpu_round.sh ${tag} tests smoke bench prof
