# Round measurement of the default bench (the GPU simulator, BASELINE configs[1])
# on the GPU box: GPU tests, smoke, the bench line (with the CPU baseline),
# kernel-trace stats, and four PMC passes (FETCH_SIZE, WRITE_SIZE, LDS/occupancy,
# instruction mix), each in its own rocprofv3 run.  Every GPU step has its own
# time limit and the script stops at the first failing step.
# usage: bash tools/sim_measure.sh [extra bench args]; outputs under gpurun_out/meas/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/meas; rm -rf $M; mkdir -p $M
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $M/gputest.log 2>&1 || { echo "pytest rc=$?"; tail -20 $M/gputest.log; exit 1; }
  tail -2 $M/gputest.log
  timeout -k 10 240 python -u __graft_entry__.py smoke > $M/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $M/smoke.log; exit 1; }
  tail -2 $M/smoke.log
fi
timeout -k 10 400 python -u bench.py "$@" > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $M/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline "$@" > $M/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $M/trace.log; exit 1; }
tail -1 $M/trace.log | cut -c1-300
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline"
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" \
    "occ SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
    "insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
  set -- $pass; name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $M/$name -o pmc --output-format csv -- python3 $B \
    > $M/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $M/$name.log; exit 1; }
  echo "pmc $name done"
done
timeout -k 10 300 python3 bench.py --mode huge > $M/huge.log 2>&1 || { echo "huge rc=$?"; tail -20 $M/huge.log; exit 1; }
tail -1 $M/huge.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $M/huge_trace -o run --output-format csv -- \
  python3 bench.py --mode huge --no-cpu-baseline > $M/huge_trace.log 2>&1 || { echo "huge trace rc=$?"; exit 1; }
timeout -k 10 600 python3 bench.py --mode placements --cmds 100 --steps 1 --warmup 0 > $M/placements.log 2>&1 \
  || { echo "placements rc=$?"; tail -20 $M/placements.log; exit 1; }
tail -1 $M/placements.log | cut -c1-300
timeout -k 10 400 python3 bench.py --mode dense-sim > $M/dense_sim.log 2>&1 || { echo "dense-sim rc=$?"; tail -20 $M/dense_sim.log; exit 1; }
tail -1 $M/dense_sim.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $M/dense_sim_trace -o run --output-format csv -- \
  python3 bench.py --mode dense-sim --no-cpu-baseline > $M/dense_sim_trace.log 2>&1 || { echo "dense-sim trace rc=$?"; exit 1; }
timeout -k 10 300 python3 bench.py --mode dense > $M/dense.log 2>&1 || { echo "dense rc=$?"; tail -20 $M/dense.log; exit 1; }
tail -1 $M/dense.log | cut -c1-300
timeout -k 10 300 python3 bench.py --mode pred > $M/pred.log 2>&1 || { echo "pred rc=$?"; tail -20 $M/pred.log; exit 1; }
tail -1 $M/pred.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $M/pred_trace -o run --output-format csv -- \
  python3 bench.py --mode pred --no-cpu-baseline > $M/pred_trace.log 2>&1 || { echo "pred trace rc=$?"; exit 1; }
find $M -name "*.csv" | sort
