"""Per-kernel GPU time of a rocprofv3 kernel trace after a marker kernel
(default: the last k_blk_fill, i.e. past a map upload), summed and divided by
a unit count: python scripts/trace_sum.py <kernel_trace.csv> <units> [marker]"""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
units = float(sys.argv[2])
marker = sys.argv[3] if len(sys.argv) > 3 else 'k_blk_fill'


def name(r):
    k = r['Kernel_Name']
    if 'rocprim' in k:
        m = re.search(r'wrapped_(\w+?)_config', k)
        return 'rocprim:' + (m.group(1) if m else '?')
    return k.split('(')[0].replace('void ', '')[-60:]


last = max([i for i, r in enumerate(rows) if marker in r['Kernel_Name']], default=-1)
acc, cnt = defaultdict(float), defaultdict(int)
for r in rows[last + 1:]:
    acc[name(r)] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cnt[name(r)] += 1
tot = sum(acc.values())
print(f"total {tot / units:.1f} us per unit over {units:g} units ({len(rows) - last - 1} launches)")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{v / units:8.1f} us {cnt[k] / units:5.1f}x  {k}")
