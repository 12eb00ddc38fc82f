# Executor-bench measurements (bench.py --mode executor): the default bench +
# kernel stats, the 100 %-conflict subset per tier, SQ counters of the group
# and lane kernels, and the lane kernel's FETCH/WRITE traffic.
# usage: bash tools/exec_measure.sh  (outputs under gpurun_out/exec/)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/exec; rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py --mode executor --steps 3 > $O/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --mode executor --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
bash tools/conflict_breakdown.sh "100:4096" "--tier 0" > $O/c100_group.txt 2>&1
bash tools/conflict_breakdown.sh "100:4096" > $O/c100_default.txt 2>&1
bash tools/pmc_tier.sh "0" --mode executor --conflicts 100 > $O/pmc_group_c100.txt 2>&1
bash tools/pmc_tier.sh "0 5" --mode executor > $O/pmc_tiers.txt 2>&1
cp -r gpurun_out/pmc_t0 gpurun_out/pmc_t5 $O/ 2>/dev/null || true
for t in 5; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f$t -o pmc --output-format csv -- python3 bench.py --mode executor --steps 1 --warmup 0 --no-cpu-baseline --tier $t > $O/f$t.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w$t -o pmc --output-format csv -- python3 bench.py --mode executor --steps 1 --warmup 0 --no-cpu-baseline --tier $t > $O/w$t.log 2>&1
done
echo done
