set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-scans 1 > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
