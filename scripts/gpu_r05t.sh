set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05t}
SLIO_LIB=_var/libslio_fe.so timeout -k 10 300 python scripts/fe_stamps.py > gpurun_out/${tag}_fe.log 2>&1 || { tail gpurun_out/${tag}_fe.log; exit 2; }
cat gpurun_out/${tag}_fe.log
