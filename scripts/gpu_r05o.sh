set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05o}
SLIO_LIB=_var/libslio_STAMP.so timeout -k 10 300 python scripts/wg_stamps.py > gpurun_out/${tag}_wg.log 2>&1 || { tail gpurun_out/${tag}_wg.log; exit 2; }
SLIO_PRIO_LATE=3 SLIO_LIB=_var/libslio_STAMP.so timeout -k 10 300 python scripts/wg_stamps.py > gpurun_out/${tag}_wg_prio.log 2>&1 || { tail gpurun_out/${tag}_wg_prio.log; exit 2; }
grep -E "^pass|WGs per CU|blocks >=" gpurun_out/${tag}_wg.log gpurun_out/${tag}_wg_prio.log
timeout -k 10 300 python scripts/ab_inproc.py - SLIO_PRIO_LATE=3 --rounds 5 > gpurun_out/${tag}_ab.log 2>&1 || { tail gpurun_out/${tag}_ab.log; exit 7; }
tail -2 gpurun_out/${tag}_ab.log
