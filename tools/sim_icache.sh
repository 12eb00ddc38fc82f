# instruction-cache counters of k_sim, fixed-geometry build vs run-time build
# (configs[1] shape, 1024 seeds x 5 rates x 200 cmds); outputs under gpurun_out/ic/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/ic; rm -rf $M; mkdir -p $M
for v in fixed generic; do
  X=""; [ $v = generic ] && X="--generic"
  timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU -d $M/$v -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --seeds 1024 --cmds 200 $X > $M/$v.log 2>&1 || { echo "$v rc=$?"; tail -20 $M/$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, glob, collections, sys
c = collections.defaultdict(float)
for f in glob.glob("gpurun_out/ic/%s/**/*counter_collection.csv" % sys.argv[1], recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_sim" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1])
for k in sorted(c): print("  %-24s %16.0f" % (k, c[k]))
PY
done
