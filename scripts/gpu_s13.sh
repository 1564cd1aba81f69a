# round-2 final tree: GPU suite, smoke, C2 bench + rocprofv3, C3 bench, live-mapping timing + rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-s13}
bash scripts/gpu_round.sh ${tag} tests smoke || exit $?
grep -q " passed" gpurun_out/${tag}_tests.log && ! grep -q "failed" gpurun_out/${tag}_tests.log || { echo "tests not green"; exit 3; }
timeout -k 10 300 python scripts/bench_aux.py mapping > gpurun_out/${tag}_aux.jsonl 2> gpurun_out/${tag}_aux.err || { tail -5 gpurun_out/${tag}_aux.err; exit 4; }
cat gpurun_out/${tag}_aux.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_auxprof -o run --output-format csv -- python3 scripts/bench_aux.py mapping > gpurun_out/${tag}_auxprof.log 2>&1 || { echo "aux prof failed"; tail -5 gpurun_out/${tag}_auxprof.log; exit 5; }
bash scripts/gpu_round.sh ${tag} bench prof benchc3
