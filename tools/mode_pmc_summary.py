"""Summarise tools/mode_pmc.sh's counter passes of one bench mode.

usage: python tools/mode_pmc_summary.py MODE DIR KERNEL_PATTERN PREFIX [bench args...]

Per dispatch of the kernels whose name contains KERNEL_PATTERN (averaged over
the main dispatches: those within 2x of the largest, so a tiered driver's small
rerun dispatches of the same kernel do not dilute it): FETCH_SIZE / WRITE_SIZE bytes, the instruction mix, waves
per CU and the issue rates.  Writes PREFIX<mode>_pmc.json (the round's record)
and profiles/pmc_<mode>.json, which the bench line of the same workload reads
(bench_pmc.py) for roofline.traffic and roofline.issue.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_dispatch(path, pat):
    """pat: a substring of the kernel names, optionally followed by
    !excluded substrings (fx::!k_synth)."""
    inc, *exc = pat.split("!")
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    names = set()
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if inc not in r["Kernel_Name"] or any(x in r["Kernel_Name"] for x in exc):
                continue
            names.add(r["Kernel_Name"])
            d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return d, names


def main():
    mode, M, pat, prefix = sys.argv[1:5]
    import bench
    import bench_pmc
    args = bench.parse(["--mode", mode] + sys.argv[5:])
    res = {"mode": mode, "kernel_pattern": pat, "workload_key": args.pmc_key}
    c = {}
    kernels = set()
    # "sum:PATTERN:STEPS": a multi-kernel step (bench.py --mode huge, the
    # quiescent-cut driver): the counters of every matching dispatch summed
    # and divided by the steps the profiled run executed (warmup + timed)
    summed = pat.startswith("sum:")
    if summed:
        pat, nsteps = pat.split(":", 1)[1].rsplit(":", 1)
        nsteps = float(nsteps)
        res["kernel_pattern"] = pat
        res["per"] = "step (%g steps profiled, every matching dispatch summed)" % nsteps
    for name in ("fetch", "write", "insts", "lds"):
        d, names = per_dispatch(os.path.join(M, name), pat)
        kernels |= names
        if d and summed:
            res["dispatches_" + name] = "%d summed" % len(d)
            for k in d:
                for ctr, v in d[k].items():
                    c[ctr] = c.get(ctr, 0.0) + v / nsteps
        elif d:
            # the main launches only: a tiered driver's rerun dispatches of the
            # same kernel over a few streams are far smaller (kept: dispatches
            # within 2x of the largest in this pass)
            size = {k: sum(v.values()) for k, v in d.items()}
            big = max(size.values())
            keep = [k for k in d if size[k] >= 0.5 * big]
            res["dispatches_" + name] = "%d of %d" % (len(keep), len(d))
            for k in keep:
                for ctr, v in d[k].items():
                    c[ctr] = c.get(ctr, 0.0) + v / len(keep)
    res["kernels"] = sorted(kernels)
    res["counters_per_dispatch"] = {k: round(v, 1) for k, v in sorted(c.items())}
    if "FETCH_SIZE" in c:
        res["read_bytes_raw"] = int(c["FETCH_SIZE"] * 1024)
        res["read_bytes_x2"] = int(c["FETCH_SIZE"] * 2048)
    if "WRITE_SIZE" in c:
        res["write_bytes"] = int(c["WRITE_SIZE"] * 1024)
    if "read_bytes_x2" in res and "write_bytes" in res:
        res["hbm_bytes_per_launch"] = res["read_bytes_x2"] + res["write_bytes"]
    if c.get("SQ_LDS_IDX_ACTIVE"):
        res["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 5)
    if c.get("GRBM_GUI_ACTIVE"):
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0  # per CU: the sum of the 8 XCDs' busy cycles / 8
        issue = {"cycles_per_cu": round(cyc)}
        if c.get("SQ_WAVE_CYCLES"):
            issue["mean_waves_per_cu"] = round(4.0 * c["SQ_WAVE_CYCLES"] / cyc / 256, 2)
            if c.get("SQ_WAIT_ANY") is not None:
                issue["wait_any_frac_of_wave_cycles"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 3)
            if c.get("SQ_BUSY_CYCLES"):
                issue["sq_busy_frac"] = round(c["SQ_BUSY_CYCLES"] / (cyc * 8), 3)
        for k, nm, units in (("SQ_INSTS_SALU", "salu_per_cu_cycle", 256), ("SQ_INSTS_VALU", "valu_per_simd_cycle", 1024),
                             ("SQ_INSTS_LDS", "lds_per_cu_cycle", 256)):
            if c.get(k):
                issue[nm] = round(c[k] / (units * cyc), 4)
        if c.get("SQ_WAVES"):
            issue["insts_per_wave"] = {k: round(c[k] / c["SQ_WAVES"]) for k in
                                       ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS") if k in c}
        res["issue"] = issue
    res["source"] = os.path.basename(prefix) + "%s_pmc.json" % mode
    res["method"] = ("rocprofv3 --pmc passes of `bench.py --mode %s --steps 1 --warmup 1 --no-cpu-baseline` "
                     "(tools/mode_pmc.sh): FETCH_SIZE, WRITE_SIZE, the instruction mix and the LDS counters "
                     "each in their own run; per dispatch of the kernels matching '%s'; traffic = FETCH_SIZE x2 "
                     "(gfx950, tools/fetch_calib.hip) + WRITE_SIZE" % (mode, pat))
    json.dump(res, open(prefix + "%s_pmc.json" % mode, "w"), indent=1)
    json.dump(res, open(os.path.join(ROOT, "profiles", "pmc_%s.json" % mode), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
