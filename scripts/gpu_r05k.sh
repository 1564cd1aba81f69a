set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05k}
for kv in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python scripts/host_gap.py --steps 400 > gpurun_out/${tag}_hostgap_kv$kv.json 2>/dev/null || exit 3
  python -c "
import json; d=json.load(open('gpurun_out/${tag}_hostgap_kv$kv.json')); m=d['stamps_median_us']
print('kernarg=$kv', 'steady', round(d['steady_median_us'],1), 'first20', round(d['first20_mean_us'],1), 'launch0', m['block_ready->launch0_returned'], 'launch0->seen', m['launch0->result_seen'], 'seen->next', m['result_seen->next_launch0'])
"
done
