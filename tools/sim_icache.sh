set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/ic; rm -rf $M; mkdir -p $M
timeout -s KILL 120 rocprofv3 -L > $M/list.txt 2>&1 || true
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU -d $M/a -o pmc --output-format csv -- \
  python3 tools/sim_perf.py --reps 1 --seeds 1024 --cmds 200 > $M/a.log 2>&1 || { echo "a rc=$?"; tail -20 $M/a.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(float)
for f in glob.glob("gpurun_out/ic/a/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_sim" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(c): print("%-24s %16.0f" % (k, c[k]))
PY
