"""Mean duration of each pass of a device-resident update from a rocprofv3
kernel trace: the search-kernel launches in order, grouped `passes` at a time
(k_search_pass instantiations only).  python scripts/pass_times.py DIR PASSES [SKIP]"""
import csv
import glob
import sys

import numpy as np

root, per = sys.argv[1], int(sys.argv[2])
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_search_pass" in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
rows = rows[skip:]
n = len(rows) // per * per
d = np.array([(e - s) / 1e3 for s, e, _ in rows[:n]]).reshape(-1, per)
gaps = np.array([(rows[k + 1][0] - rows[k][1]) / 1e3 for k in range(n - 1)] + [0.0]).reshape(-1, per)
print(f"{d.shape[0]} groups of {per} launches")
for j in range(per):
    print(f"pass {j}: mean {d[:, j].mean():7.2f} us  median {np.median(d[:, j]):7.2f}  gap before next {np.median(gaps[:, j]):6.2f}")
