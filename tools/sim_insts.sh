# Instruction mix of k_sim on the configs[1] bench (one PMC pass):
# bash tools/sim_insts.sh [bench args]; prints SALU / VALU per wave and the
# scalar unit's issue rate (SALU per CU cycle).  Output under gpurun_out/insts/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/insts; rm -rf $M; mkdir -p $M
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  -d $M/p -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $M/log 2>&1 \
  || { echo "rc=$?"; tail -20 $M/log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
c = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/insts/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_sim" in r["Kernel_Name"]:
            c[r["Counter_Name"]] += float(r["Counter_Value"])
w = c["SQ_WAVES"]; cyc = c["GRBM_GUI_ACTIVE"]
print("waves %d  SALU/wave %.2fM  VALU/wave %.2fM  BR/wave %.2fM  LDS/wave %.2fM" % (w, c["SQ_INSTS_SALU"]/w/1e6, c["SQ_INSTS_VALU"]/w/1e6, c["SQ_INSTS_BRANCH"]/w/1e6, c["SQ_INSTS_LDS"]/w/1e6))
print("SALU per CU cycle %.3f  VALU per SIMD cycle %.3f  (GRBM cycles %.3g)" % (c["SQ_INSTS_SALU"]/cyc/256, c["SQ_INSTS_VALU"]/cyc/1024, cyc))
PY
