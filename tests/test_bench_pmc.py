"""bench_pmc: the counter record of a bench mode reaches the line's roofline
block only for its own workload, with traffic, LDS bank conflicts and wave
occupancy (north_star's rocprof figures).  CPU only."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench_pmc  # noqa: E402


def test_attach_copies_traffic_conflicts_and_occupancy():
    pm = {"mode": "sim", "source": "x.json", "hbm_bytes_per_launch": 300, "read_bytes_x2": 200,
          "write_bytes": 100, "lds_bank_conflict_frac": 0.0019, "kernel_pattern": "k_sim<",
          "issue": {"mean_waves_per_cu": 14.89, "salu_per_cu_cycle": 0.69}}
    roof = bench_pmc.attach({}, pm, 1000)
    assert roof["traffic"] == 300 and roof["traffic_over_alg"] == 0.3
    assert roof["lds_bank_conflict_frac"] == 0.0019
    assert roof["mean_waves_per_cu"] == 14.89
    assert roof["issue"]["salu_per_cu_cycle"] == 0.69


def test_record_of_another_workload_is_not_used(tmp_path, monkeypatch):
    args = argparse.Namespace(mode="sim", seeds=4096, steps=3)
    other = argparse.Namespace(mode="sim", seeds=1024, steps=3)
    monkeypatch.setattr(bench_pmc, "ROOT", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    with open(tmp_path / "profiles" / "pmc_sim.json", "w") as f:
        json.dump({"workload_key": bench_pmc.workload_key(args), "hbm_bytes_per_launch": 1}, f)
    assert bench_pmc.load("sim", args) is not None
    assert bench_pmc.load("sim", other) is None
    # the step count does not change a launch's work
    assert bench_pmc.load("sim", argparse.Namespace(mode="sim", seeds=4096, steps=7)) is not None
