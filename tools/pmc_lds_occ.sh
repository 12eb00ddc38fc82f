# One PMC pass over the default bench for LDS bank conflicts and wave occupancy
# (BASELINE asks for both next to the HBM roofline).  Counters fit one pass:
# 6 SQ + 2 GRBM.  usage: bash tools/pmc_lds_occ.sh [bench args]; output gpurun_out/meas/occ
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/meas; mkdir -p $M
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $M/occ -o pmc --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $M/occ.log 2>&1 \
  || { echo "occ rc=$?"; tail -20 $M/occ.log; exit 1; }
find $M/occ -name "*.csv" | sort
