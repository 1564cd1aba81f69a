"""Summarise a rocprofv3 kernel/memcpy trace: per-kernel mean duration and the
mean gap before each kernel (device idle time) over the last N steps."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
rows = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
for f in glob.glob(f"{root}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
rows.sort()
tail = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -400:]
dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
prev = None
for s, e, n in tail:
    dur[n] += e - s
    cnt[n] += 1
    if prev is not None:
        gap[n] += max(0, s - prev)
    prev = e
span = tail[-1][1] - tail[0][0]
print(f"span {span/1e3:.1f} us over {len(tail)} ops")
for n in sorted(dur, key=lambda k: -dur[k]):
    print(f"{cnt[n]:5d}  dur {dur[n]/cnt[n]/1e3:8.2f} us  gap-before {gap[n]/cnt[n]/1e3:8.2f} us  {n}")
