set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05v}
bash scripts/gpu_r05r.sh $tag || exit $?
SLIO_LIB=_var/libslio_fe.so timeout -k 10 300 python scripts/fe_stamps.py > gpurun_out/${tag}_fe.log 2>&1 || { tail gpurun_out/${tag}_fe.log; exit 7; }
grep -v amdgpu.ids gpurun_out/${tag}_fe.log
