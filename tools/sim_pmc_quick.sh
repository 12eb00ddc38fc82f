# Two PMC passes (instruction mix, issue/LDS waits) over tools/sim_perf.py.
# usage: bash tools/sim_pmc_quick.sh [sim_perf args]; output gpurun_out/q/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/q; rm -rf $M; mkdir -p $M
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY \
  SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $M/a -o pmc --output-format csv -- \
  python3 tools/sim_perf.py --reps 1 "$@" > $M/a.log 2>&1 || { echo "a rc=$?"; tail -20 $M/a.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES \
  SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d $M/b -o pmc --output-format csv -- \
  python3 tools/sim_perf.py --reps 1 "$@" > $M/b.log 2>&1 || { echo "b rc=$?"; tail -20 $M/b.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(float)
for f in glob.glob("gpurun_out/q/*/**/*counter_collection.csv", recursive=True) + glob.glob("gpurun_out/q/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_sim" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
w = c["SQ_WAVES"] or 1
for k in sorted(c):
    print("%-24s %16.0f  per wave %14.0f" % (k, c[k], c[k] / w))
PY
