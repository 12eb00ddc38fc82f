# Two SQ PMC passes (instruction mix, wait/active split) per tier on one bench variant.
# usage: bash tools/pmc_tier.sh "0 5" [bench args]; summaries in gpurun_out/pmc_t<tier>/summary.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tiers=$1; shift
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
for t in $tiers; do
  OUT=gpurun_out/pmc_t$t; rm -rf $OUT; mkdir -p $OUT
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P -d $OUT/p$i -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --tier $t "$@" > $OUT/p$i.log 2>&1
  done
  python3 tools/pmc_summary.py $OUT k_graph > $OUT/summary.txt
  echo "== tier $t"; cat $OUT/summary.txt
done
