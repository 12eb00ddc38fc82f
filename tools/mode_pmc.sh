# Counter passes of one bench mode's dominant kernel (rocprofv3 --pmc, one
# counter group per run, each under its own time limit; the script stops at the
# first failing step).  usage:
#   [PMC_TAG=name] bash tools/mode_pmc.sh MODE KERNEL_PATTERN [bench args]
# outputs under gpurun_out/pmc_<PMC_TAG or mode>/; summarise with tools/mode_pmc_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
MODE=$1; PAT=$2; shift 2
M=gpurun_out/pmc_${PMC_TAG:-$MODE}; rm -rf $M; mkdir -p $M
B="bench.py --mode $MODE --steps 1 --warmup 1 --no-cpu-baseline $@"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $M/trace -o run --output-format csv -- python3 $B \
  > $M/trace.log 2>&1 || { echo "$MODE trace rc=$?"; tail -20 $M/trace.log; exit 1; }
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" \
    "insts SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
    "lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_COUNT"; do
  set -- $pass; name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" -d $M/$name -o pmc --output-format csv -- python3 $B \
    > $M/$name.log 2>&1 || { echo "$MODE $name rc=$?"; tail -20 $M/$name.log; exit 1; }
  echo "$MODE pmc $name done"
done
