# round-5: are the simulators instruction-cache bound?  the counters the box
# offers, then one pass of the instruction-fetch counters on dense-sim and sim
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5ic; mkdir -p $M
timeout -k 10 120 rocprofv3 -L > $M/avail.txt 2>&1 || { echo "list rc=$?"; tail -5 $M/avail.txt; exit 1; }
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_SMEM\|SQ_WAIT_INST_ANY\|SQ_INST_CYCLES_SALU\|SQ_ACTIVE_INST_SCA\|SQ_INSTS_BRANCH" $M/avail.txt | sort -u | tee $M/found.txt
C=$(grep -o "SQC_ICACHE_HITS\|SQC_ICACHE_MISSES\|SQC_ICACHE_MISSES_DUPLICATE\|SQ_IFETCH" $M/found.txt | sort -u | head -4 | tr '\n' ' ')
[ -n "$C" ] || { echo "no icache counters"; exit 0; }
for mode in dense-sim sim; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $M/$mode -o pmc --output-format csv -- python3 bench.py --mode $mode --steps 1 --warmup 0 --no-cpu-baseline \
    > $M/$mode.log 2>&1 || { echo "$mode rc=$?"; tail -5 $M/$mode.log; exit 1; }
  echo "$mode done"
done
