# The lane tier's traffic and the executor bench step: WRITE_SIZE / FETCH_SIZE
# of k_graph_lane (tier 5, one launch over the configs[1]-shaped batch), each in
# its own rocprofv3 pass, and one default executor bench run.
# usage: bash tools/lane_traffic.sh TAG   (outputs under gpurun_out/lt_TAG/)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lt_$1; rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py --mode executor --steps 3 > $O/bench.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w5 -o pmc --output-format csv -- python3 bench.py --mode executor --steps 1 --warmup 0 --no-cpu-baseline --tier 5 > $O/w5.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f5 -o pmc --output-format csv -- python3 bench.py --mode executor --steps 1 --warmup 0 --no-cpu-baseline --tier 5 > $O/f5.log 2>&1
python3 - $O <<'PY'
import csv, collections, glob, json, sys
O = sys.argv[1]
for name in ("w5", "f5"):
    d = collections.defaultdict(float)
    for f in glob.glob(O + "/" + name + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_graph_lane" in r["Kernel_Name"]:
                d[r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(name, "k_graph_lane GB per dispatch:", [round(v * 1024 / 1e9, 3) for v in d.values()])
b = json.loads(open(O + "/bench.log").read().strip().splitlines()[-1])
print("bench value %.3f G ms_per_step %s kernel_ms_avg %s" % (b["value"] / 1e9, b["ms_per_step"], b["roofline"].get("kernel_ms_avg")))
PY
