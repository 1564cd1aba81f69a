# diagnostic / ablation builds into agi_lidar_slam_amd/_abl: bash scripts/build_abl.sh NAME "-DFLAG ..." [NAME "FLAGS"]...
# SRC=<dir> builds from another copy of csrc (e.g. an earlier commit's, for an A/B)
cd "$(dirname "$0")/.."
mkdir -p agi_lidar_slam_amd/_abl
S=${SRC:-agi_lidar_slam_amd/csrc}
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math $2 -I include \
    -I agi_lidar_slam_amd/csrc $S/slio_device.hip $S/slio_ikf.cpp $S/slio_imu.cpp $S/slio_s2m.cpp $S/slio_lio.hip \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o agi_lidar_slam_amd/_abl/libslio_$1.so &
  shift 2
done
wait
