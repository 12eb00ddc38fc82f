"""Summarise rocprofv3 --pmc CSVs: per kernel (name substring), mean per dispatch of each counter."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_graph_exec"
vals = defaultdict(list)
for f in sorted(glob.glob(root + "/p*/pmc_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
for c in sorted(vals):
    v = vals[c]
    print("%-28s n=%d mean=%.4g" % (c, len(v), sum(v) / len(v)))
