# usage: [OUT=dir] bash scripts/build_variant.sh <name> [-DDEFINE ...]
# builds ${OUT:-agi_lidar_slam_amd/_abl}/libslio_<name>.so from the current sources
# with extra defines (diagnostic or A/B builds; the product library is build.py's).
# _abl is not shipped to the GPU box (.gpurunignore): for a GPU run build with
# OUT=_var (git-ignored, shipped; empty it when done) and bind the build with
# scripts/variant.py
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=agi_lidar_slam_amd/_abl/obj_$name
mkdir -p $out ${OUT:-agi_lidar_slam_amd/_abl}
tag=$(python3 -c "from agi_lidar_slam_amd import build; print(build.source_hash())")
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -DSLIO_SOURCE_HASH=\"$tag\" -Iinclude $*"
pids=()
for s in slio_device.hip slio_ikf.cpp slio_imu.cpp slio_s2m.cpp slio_lio.hip; do
  /opt/rocm/bin/hipcc $F -c agi_lidar_slam_amd/csrc/$s -o $out/$s.o 2>$out/$s.err & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
  -o ${OUT:-agi_lidar_slam_amd/_abl}/libslio_$name.so
rm -rf $out
echo ${OUT:-agi_lidar_slam_amd/_abl}/libslio_$name.so
