"""Summarise rocprofv3 PMC passes for k_search_pass into profiles/<name>.json.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB counters x 1024):
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads
(MI355X_MICROARCH.md §HBM); the search pass reads 16-B float4 per lane, the
calibrated width.  Infinity-Cache hits are counted as fetches."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(out_json, *dirs):
    vals = defaultdict(list)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_search_pass" in r.get("Kernel_Name", ""):
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    fetch = mean.get("FETCH_SIZE")
    write = mean.get("WRITE_SIZE")
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from agi_lidar_slam_amd import build
    res = {
        "kernel": "k_search_pass",
        # bench.py attaches hbm_bytes_per_launch only to runs of the library
        # built from these sources
        "source_hash": build.source_hash(),
        "map_points": 10_000_000,
        "scan_points": 100_000,
        "counters_mean_per_launch": mean,
        "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None else None,
        "note": "2*FETCH_SIZE+WRITE_SIZE (KiB) per launch, gfx950 FETCH_SIZE halving corrected",
    }
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        res["l2_hit_rate"] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:])
