set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/ab_bench.sh r3j 3 agi_lidar_slam_amd/_abl/libslio_B.so agi_lidar_slam_amd/_abl/libslio_F.so
