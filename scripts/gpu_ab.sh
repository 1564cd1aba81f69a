# one GPU call: the C2-path GPU tests, then an in-process A/B of update
# switches and the C2 pass timeline under rocprofv3 -> gpurun_out/<tag>_*
#   bash scripts/gpu_ab.sh <tag> "<pytest -k expr>" <ab configs...>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; kexpr=$2; shift 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_comm.py -m gpu -x -v --timeout 300 --timeout-method thread -k "$kexpr" > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 400 python scripts/ab_inproc.py "$@" > gpurun_out/${tag}_ab.log 2>&1 || { tail -20 gpurun_out/${tag}_ab.log; exit 4; }
cat gpurun_out/${tag}_ab.log | tail -${#}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_c2 -o run -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/${tag}_bench_c2.json 2>/dev/null || exit 5
python scripts/pass_times.py gpurun_out/${tag}_prof_c2 4 40 > gpurun_out/${tag}_c2_pass_times.txt && cat gpurun_out/${tag}_c2_pass_times.txt
