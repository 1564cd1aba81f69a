# round 3, session start: baseline bench, search-pass stamps (init / GT pose), filter-step stamps
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || { echo bench failed; tail gpurun_out/r3a_bench.err; exit 4; }
cat gpurun_out/r3a_bench.json
for pose in init gt; do
  STAMP_POSE=$pose LPQS=2 SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_STAMP.so timeout -k 10 200 python scripts/stamps.py > gpurun_out/r3a_stamps_$pose.log 2>&1 || { echo stamps failed; tail gpurun_out/r3a_stamps_$pose.log; exit 5; }
  mv gpurun_out/stamps_2_100000.npz gpurun_out/r3a_stamps_$pose.npz
  grep -v amdgpu.ids gpurun_out/r3a_stamps_$pose.log
done
SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_SOLVE.so timeout -k 10 200 python scripts/solve_stamps.py > gpurun_out/r3a_solve.log 2>&1 || { echo solve failed; tail gpurun_out/r3a_solve.log; exit 6; }
grep -v amdgpu.ids gpurun_out/r3a_solve.log
