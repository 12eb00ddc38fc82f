# k_graph_lane drift bound sweep: time (tier 5 alone and the default split
# tier) and FETCH/WRITE per launch.  usage: bash tools/lane_drift.sh "0 1 2 4"
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/drift; rm -rf $O; mkdir -p $O
for d in $1; do
  export FX_LANE_DRIFT=$d
  timeout -k 10 200 python bench.py --mode executor --steps 3 --no-cpu-baseline --tier 5 > $O/t5_$d.log 2>&1
  timeout -k 10 200 python bench.py --mode executor --steps 3 --no-cpu-baseline > $O/t6_$d.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f$d -o pmc --output-format csv -- python3 bench.py --mode executor --steps 1 --warmup 0 --no-cpu-baseline --tier 5 > $O/f$d.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w$d -o pmc --output-format csv -- python3 bench.py --mode executor --steps 1 --warmup 0 --no-cpu-baseline --tier 5 > $O/w$d.log 2>&1
  python3 - $O $d <<'PY'
import csv, glob, json, sys, collections
O, d = sys.argv[1], sys.argv[2]
def kern(tag):
    out = collections.defaultdict(float)
    for f in glob.glob("%s/%s%s/**/*counter_collection.csv" % (O, tag, d), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_graph_lane" in r["Kernel_Name"]:
                out[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(out.values()) / max(1, len(out))
def line(f):
    return json.loads(open(f).read().strip().splitlines()[-1])
a, b = line("%s/t5_%s.log" % (O, d)), line("%s/t6_%s.log" % (O, d))
print("drift %s: tier5 %.1f ms (lane %.1f ms), split %.1f ms %s; lane FETCH %.2f GB raw, WRITE %.2f GB" % (
    d, a["ms_per_step"], a["roofline"].get("kernel_ms_avg", 0), b["ms_per_step"],
    b["roofline"].get("per_kernel_ms_avg"), kern("f") / 1e6, kern("w") / 1e6))
PY
done
