set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r06t}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_gpu_tests.log; exit 3; }
tail -3 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 4; }
tail -2 gpurun_out/${tag}_smoke.log
