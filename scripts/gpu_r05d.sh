set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05d}
timeout -k 10 300 python scripts/cert_probe.py > gpurun_out/${tag}_probe.log 2>&1 || { tail gpurun_out/${tag}_probe.log; exit 3; }
cat gpurun_out/${tag}_probe.log
SLIO_NO_KNN_CERT=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_prof_cert -o run -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline --timing-steps 1 > gpurun_out/${tag}_b1.json 2>/dev/null || exit 4
python scripts/pass_times.py gpurun_out/${tag}_prof_cert 4 40
