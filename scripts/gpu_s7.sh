# refinement lanes-per-query A/B (8 -> 4 -> 2 lanes as a chunk's refining
# queries grow), stamps of pass 0 for both, then the GPU suite on the in-tree lib
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s7}
A=agi_lidar_slam_amd/_abl
cp agi_lidar_slam_amd/libslio.so $A/libslio_intree.so || exit 3
bash scripts/ab_bench.sh ${tag} $A/libslio_lazy.so $A/libslio_rl8.so $A/libslio_rl4.so || exit 3
for v in STAMP STAMPrl4; do
  SLIO_LIB=$A/libslio_$v.so LPQS=2 timeout -k 10 180 python scripts/stamps.py > gpurun_out/${tag}_stamps_$v.log 2>&1 || { echo "stamps $v failed"; tail -5 gpurun_out/${tag}_stamps_$v.log; exit 5; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${tag}_stamps_$v.log | tail -14
done
cp $A/libslio_intree.so agi_lidar_slam_amd/libslio.so || exit 3
bash scripts/gpu_round.sh ${tag} tests
