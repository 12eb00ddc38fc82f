"""Summarise the PMC passes of tools/sim_measure.sh for the simulator kernel.

usage: python tools/sim_pmc_summary.py gpurun_out/meas profiles/<round>_ [bench args...]

Writes <prefix>sim_pmc.json (per-dispatch counters of k_sim averaged over its
dispatches, with derived figures) and profiles/sim_traffic_latest.json (the
per-launch memory-side traffic that bench.py reports as roofline.traffic for
the same workload key).  Derived figures:
* read bytes: FETCH_SIZE (KB) x 1024, raw, and x 2 (the gfx950 correction that
  MI355X_MICROARCH.md documents for wide coalesced reads; k_sim's reads are
  narrow, so the raw figure is the one to trust and both are printed);
* write bytes: WRITE_SIZE (KB) x 1024;
* lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* mean_waves_per_cu = 4 SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs) / 256 CUs;
* per-wave instruction mix and the issue split ACTIVE / WAIT_INST / WAIT of
  SQ_WAVE_CYCLES.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNEL = "k_sim"


def per_dispatch(path):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "::" + KERNEL + "(" not in r["Kernel_Name"] and "::" + KERNEL + "<" not in r["Kernel_Name"]:
                continue
            d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return d


def mean(d):
    out = collections.defaultdict(float)
    for c in d.values():
        for k, v in c.items():
            out[k] += v / len(d)
    return out


def main():
    M, prefix = sys.argv[1], sys.argv[2]
    import bench
    import bench_sim
    args = bench.parse(sys.argv[3:])
    if args.cmds is None:
        args.cmds = 1000  # bench_sim.main_sim default
    key = bench_sim.sim_key(args)
    res = {"kernel": KERNEL, "workload_key": key}
    c = {}
    for name in ("fetch", "write", "occ", "insts"):
        d = per_dispatch(os.path.join(M, name))
        if d:
            res["dispatches_" + name] = len(d)
            c.update(mean(d))
    res["counters_per_dispatch"] = {k: round(v, 1) for k, v in sorted(c.items())}
    if "FETCH_SIZE" in c:
        res["read_bytes_raw"] = int(c["FETCH_SIZE"] * 1024)
        res["read_bytes_x2"] = int(c["FETCH_SIZE"] * 2048)
    if "WRITE_SIZE" in c:
        res["write_bytes"] = int(c["WRITE_SIZE"] * 1024)
    if c.get("SQ_LDS_IDX_ACTIVE"):
        res["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 5)
    if c.get("GRBM_GUI_ACTIVE"):
        res["mean_waves_per_cu"] = round(4.0 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8) / 256, 2)
        res["occupancy_frac"] = round(res["mean_waves_per_cu"] / 16.0, 3)  # 4 waves/SIMD (k_sim<1,1,4>) x 4 SIMDs
    if c.get("SQ_WAVES") or c.get("SQ_INSTS_VALU"):
        waves = c.get("SQ_WAVES") or 0
        if waves:
            res["insts_per_wave"] = {k: round(c[k] / waves) for k in
                                     ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
                                      "SQ_INSTS_LDS") if k in c}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc and "SQ_ACTIVE_INST_ANY" in c:
            res["wave_cycle_split"] = {"active_inst": round(c["SQ_ACTIVE_INST_ANY"] / wc, 3),
                                       "wait_inst": round(c["SQ_WAIT_INST_ANY"] / wc, 3),
                                       "wait_any": round(c["SQ_WAIT_ANY"] / wc, 3)}
    if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_INSTS_SALU"):
        # issue rates: GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs, so
        # cycles per CU = GRBM_GUI_ACTIVE / 8; the CU's scalar unit issues at
        # most one SALU instruction per cycle (the arbiter serves one SIMD per
        # cycle), each SIMD at most one VALU instruction per cycle
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        res["issue"] = {
            "cycles_per_cu": round(cyc),
            "salu_per_cu_cycle": round(c["SQ_INSTS_SALU"] / (256 * cyc), 4),
            "valu_per_simd_cycle": round(c["SQ_INSTS_VALU"] / (1024 * cyc), 4),
            "all_per_cu_cycle": round(sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
                                                                   "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"))
                                      / (256 * cyc), 4)}
    json.dump(res, open(prefix + "sim_pmc.json", "w"), indent=1)
    if "read_bytes_raw" in res and "write_bytes" in res and key:
        tj = {"workload_key": key, "kernel": KERNEL,
              "hbm_bytes_per_launch": res["read_bytes_raw"] + res["write_bytes"],
              "read_bytes_raw": res["read_bytes_raw"], "read_bytes_x2": res["read_bytes_x2"],
              "write_bytes": res["write_bytes"], "issue": res.get("issue"),
              "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
                        "(tools/sim_measure.sh), per k_sim dispatch; raw FETCH_SIZE (k_sim's loads are "
                        "narrow, not the wide streaming reads the x2 gfx950 correction is documented for; "
                        "read_bytes_x2 gives the corrected figure beside it)",
              "source": os.path.basename(prefix) + "sim_pmc.json"}
        json.dump(tj, open(os.path.join(ROOT, "profiles", "sim_traffic_latest.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
