# Round measurement on the GPU box: parity tests, smoke, default bench (with the
# CPU baseline), kernel-trace stats and the two HBM-traffic PMC passes of the
# default bench.  Each GPU step has its own time limit; the script stops at the
# first failing step.
# usage: bash tools/round_measure.sh [extra bench args]; outputs under gpurun_out/meas/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/meas; rm -rf $M; mkdir -p $M
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $M/gputest.log 2>&1 || { echo "pytest rc=$?"; tail -20 $M/gputest.log; exit 1; }
tail -2 $M/gputest.log
timeout -k 10 240 python -u __graft_entry__.py smoke > $M/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $M/smoke.log; exit 1; }
tail -1 $M/smoke.log
timeout -k 10 300 python bench.py "$@" > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $M/bench.log; exit 1; }
tail -1 $M/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $M/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline "$@" > $M/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $M/trace.log; exit 1; }
tail -1 $M/trace.log
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $M/fetch -o pmc --output-format csv -- python3 $B "$@" \
  > $M/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -20 $M/fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $M/write -o pmc --output-format csv -- python3 $B "$@" \
  > $M/write.log 2>&1 || { echo "write rc=$?"; tail -20 $M/write.log; exit 1; }
find $M -name "*.csv" | sort
