set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r3f}
SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_SOLVE.so timeout -k 10 200 python scripts/solve_stamps.py > gpurun_out/${tag}_solve.log 2>&1 || { echo solve failed; tail gpurun_out/${tag}_solve.log; exit 6; }
grep -v amdgpu.ids gpurun_out/${tag}_solve.log
