# one GPU call: the C2-path GPU tests, a bench.py A/B over library builds
# (scripts/ab_bench.sh), then one WRITE_SIZE PMC pass of k_search_pass per
# build -> gpurun_out/<tag>_*
#   bash scripts/gpu_store_ab.sh <tag> lib1.so lib2.so ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused or c2_full or knn_cert or reference_gain" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 3; }
tail -1 gpurun_out/${tag}_tests.log
bash scripts/ab_bench.sh $tag 3 "$@" || exit 4
for lib in "$@"; do
  n=$(basename $lib .so)
  MODE=update REPS=10 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_search_pass -d gpurun_out/${tag}_w_$n -o pmc --output-format csv -- python3 scripts/variant.py $lib scripts/run_search.py > gpurun_out/${tag}_w_$n.log 2>&1 || { echo "pmc $n failed"; tail -3 gpurun_out/${tag}_w_$n.log; exit 6; }
  PMC_KERNELS=k_search_pass python3 scripts/pmc_traffic.py gpurun_out/${tag}_w_$n.json gpurun_out/${tag}_w_$n > /dev/null && python3 -c "import json; d=json.load(open('gpurun_out/${tag}_w_$n.json')); print('$n WRITE_SIZE KiB/launch', round(d['counters_mean_per_launch']['WRITE_SIZE']))"
done
