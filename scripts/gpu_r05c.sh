set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
true

SLIO_NO_KNN_CERT=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05c_prof_cert -o run -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline --timing-steps 1 > gpurun_out/r05c_b1.json 2>/dev/null || exit 4
SLIO_NO_KNN_CERT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05c_prof_full -o run -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline --timing-steps 1 > gpurun_out/r05c_b2.json 2>/dev/null || exit 5
python scripts/pass_times.py gpurun_out/r05c_prof_cert 4 40
python scripts/pass_times.py gpurun_out/r05c_prof_full 4 40
