"""The measurement tooling behind bench.py's roofline.traffic (CPU only):
scripts/pmc_traffic.py's per-kernel PMC summary and the source-hash gate that
keeps a summary from being attached to a library built from other sources."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _counter_csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_summary_sums_kernels(tmp_path):
    d1, d2 = tmp_path / "p1", tmp_path / "p2"
    # two passes (FETCH_SIZE, WRITE_SIZE), two launches of each kernel
    _counter_csv(str(d1 / "x_counter_collection.csv"), [
        {"Kernel_Name": "void slio::lio::k_fe_pick<0, 512>(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 10},
        {"Kernel_Name": "void slio::lio::k_fe_pick<0, 512>(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 30},
        {"Kernel_Name": "void slio::lio::k_fe_ring<0, 2048>(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 100},
        {"Kernel_Name": "slio::lio::k_lio_fill(...)", "Counter_Name": "FETCH_SIZE", "Counter_Value": 999},
    ])
    _counter_csv(str(d2 / "x_counter_collection.csv"), [
        {"Kernel_Name": "void slio::lio::k_fe_pick<0, 512>(...)", "Counter_Name": "WRITE_SIZE", "Counter_Value": 4},
        {"Kernel_Name": "void slio::lio::k_fe_ring<0, 2048>(...)", "Counter_Name": "WRITE_SIZE", "Counter_Value": 6},
    ])
    out = tmp_path / "t.json"
    env = dict(os.environ, PMC_KERNELS="k_fe_pick,k_fe_ring", PMC_WORKLOAD="c3")
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), str(out), str(d1), str(d2)],
                   check=True, env=env, capture_output=True)
    res = json.load(open(out))
    assert res["workload"] == "c3"
    # per-launch means summed over the two kernels: FETCH 20 + 100, WRITE 4 + 6 (KiB)
    assert res["counters_mean_per_launch"]["FETCH_SIZE"] == 120
    assert res["counters_mean_per_launch"]["WRITE_SIZE"] == 10
    assert res["hbm_bytes_per_launch"] == (2 * 120 + 10) * 1024
    from agi_lidar_slam_amd import build
    assert res["source_hash"] == build.source_hash()


def test_frontend_traffic_gated_by_sources(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    from agi_lidar_slam_amd import build
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    path = tmp_path / "profiles" / "lego_traffic.json"
    json.dump({"workload": "lego", "source_hash": build.source_hash(), "hbm_bytes_per_launch": 1234.0},
              open(path, "w"))
    assert bench.frontend_traffic("lego") == 1234.0
    assert bench.frontend_traffic("c3") is None  # no summary for that workload
    json.dump({"workload": "lego", "source_hash": "0" * 16, "hbm_bytes_per_launch": 1234.0}, open(path, "w"))
    assert bench.frontend_traffic("lego") is None  # other sources: not attached
