"""Per-dispatch FETCH_SIZE / WRITE_SIZE of the executor kernels from the two PMC
passes of tools/round_measure.sh, and the per-launch HBM traffic JSON that
bench.py reports as roofline.traffic.
usage: python tools/traffic_summary.py gpurun_out/meas [profiles/<round>_] [--json profiles/traffic_latest.json]"""
import csv
import json
import sys
from collections import defaultdict

EXEC = ("k_split_score", "k_split_plan", "k_graph_lane", "k_graph_group")
M = sys.argv[1]
prefix = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
jpath = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
kb = {}
for name, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    per, names = defaultdict(float), {}
    for r in csv.DictReader(open("%s/%s/pmc_counter_collection.csv" % (M, name))):
        if any(k in r["Kernel_Name"] for k in EXEC):
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
    if prefix:
        with open("%spmc_%s.csv" % (prefix, ctr.lower()), "w") as f:
            f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value_KB_summed\n")
            for d in sorted(per, key=int):
                f.write('%s,"%s",%s,%s\n' % (d, names[d], ctr, per[d]))
    launches = max(1, len([d for d in per if "k_graph_group" in names[d] or "k_graph_lane" in names[d]
                           and not any("k_graph_group" in v for v in names.values())]))
    for d in sorted(per, key=int):
        print("%-10s %-5s %-45s %12.0f KB" % (ctr, d, names[d][:45], per[d]))
    kb[ctr] = sum(per.values()) / launches
rd, wr = kb["FETCH_SIZE"] * 1024 * 2, kb["WRITE_SIZE"] * 1024
print("per launch: read %.2f GB (FETCH_SIZE x2), write %.2f GB, total %.2f GB" % (rd / 1e9, wr / 1e9, (rd + wr) / 1e9))
if jpath:
    j = {"workload_key": "n5_s4096_c0-2-10-50-100_m1000_w8_y30_seed20250213_b-1_t-1",
         "kernel": "k_graph_group||k_graph_lane",
         "hbm_bytes_per_launch": int(rd + wr), "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wr),
         "fetch_size_kb": kb["FETCH_SIZE"], "write_size_kb": kb["WRITE_SIZE"],
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/round_measure.sh), "
                   "summed over the dispatches of one split-tier executor launch (k_split_score, k_split_plan, "
                   "k_graph_lane, k_graph_group); FETCH_SIZE x2 for 16 B/lane loads on gfx950 "
                   "(MI355X_MICROARCH.md, HBM section); KB units. FETCH_SIZE counts memory-side L2 requests, "
                   "Infinity-Cache hits included, so it bounds HBM reads from above",
         "round": 1}
    json.dump(j, open(jpath, "w"), indent=1)
