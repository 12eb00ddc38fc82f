# Instruction mix and LDS waits of k_graph_wide on the dense executor bench
# (bench.py --mode dense, BASELINE configs[3] streams), two PMC passes plus a
# kernel trace: bash tools/pmc_dense.sh [bench args]; output under gpurun_out/pmcd/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/pmcd; rm -rf $M; mkdir -p $M
B="bench.py --mode dense --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $M/trace -o run --output-format csv -- python3 $B "$@" \
  > $M/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $M/trace.log; exit 1; }
tail -1 $M/trace.log | cut -c1-300
for pass in "insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
    "waits SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES"; do
  set -- $pass; name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $M/$name -o pmc --output-format csv -- python3 $B \
    > $M/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $M/$name.log; exit 1; }
  echo "pmc $name done"
done
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(float)
for f in glob.glob("gpurun_out/pmcd/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_graph_wide" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(c):
    print("%-22s %.4g" % (k, c[k]))
PY
