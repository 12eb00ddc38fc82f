"""Summarise the LDS / occupancy PMC pass (tools/pmc_lds_occ.sh) per kernel.

usage: python tools/occ_summary.py gpurun_out/meas/occ/pmc_counter_collection.csv > profiles/<round>_lds_occupancy.json

Derived figures (per kernel, summed over its dispatches):
* lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over
  all LDS-array cycles, MI355X_MICROARCH.md "LDS");
* mean_waves_per_cu = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8) / 256 — SQ_WAVE_CYCLES
  counts wave-resident quad-cycles summed over all CUs, GRBM_GUI_ACTIVE is summed over
  the 8 XCDs by rocprofv3; 256 CUs.  (An estimate: gfx950 has no derived-counter table
  in ROCm 7.2, so the unit assumptions are the gfx94x ones.)
* occupancy_frac = mean_waves_per_cu / (waves per SIMD the kernel's resources allow * 4).
"""
import collections
import csv
import json
import sys

CUS = 256
XCDS = 8
# waves per SIMD allowed by each kernel's VGPR/LDS budget (make resource-usage)
WAVES_PER_SIMD = {"k_graph_group": 5, "k_graph_lane": 2, "k_metrics": 8}


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not name.startswith(("fx::", "void fx::")):
            continue
        key = name.split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    out = {}
    for k, c in agg.items():
        gui = c["GRBM_GUI_ACTIVE"] / XCDS
        waves = 4.0 * c["SQ_WAVE_CYCLES"] / gui / CUS if gui else 0.0
        d = {
            "dispatches": len(disp[k]),
            "counters": {n: int(v) for n, v in sorted(c.items())},
            "lds_bank_conflict_frac": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
                                       if c["SQ_LDS_IDX_ACTIVE"] else 0.0),
            "mean_waves_per_cu": round(waves, 2),
        }
        if k in WAVES_PER_SIMD:
            d["occupancy_frac"] = round(waves / (4 * WAVES_PER_SIMD[k]), 3)
        out[k] = d
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
