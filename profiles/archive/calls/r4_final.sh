# Round-4 closing checks on the GPU box: every GPU test, smoke, the handle and
# executor bench lines.  Each step under its own limit; stops at the first failure.
# usage: bash profiles/archive/calls/r4_final.sh   (outputs under gpurun_out/fin/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/fin; rm -rf $M; mkdir -p $M
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $M/gputest.log 2>&1 || { echo "pytest rc=$?"; tail -20 $M/gputest.log; exit 1; }
tail -2 $M/gputest.log
timeout -k 10 240 python -u __graft_entry__.py smoke > $M/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $M/smoke.log; exit 1; }
tail -2 $M/smoke.log
timeout -k 10 300 python -u bench.py --mode handle > $M/handle.log 2>&1 || { echo "handle rc=$?"; tail -20 $M/handle.log; exit 1; }
tail -1 $M/handle.log | cut -c1-300
timeout -k 10 300 python -u bench.py --mode executor > $M/executor.log 2>&1 || { echo "executor rc=$?"; tail -20 $M/executor.log; exit 1; }
tail -1 $M/executor.log | cut -c1-300
timeout -k 10 400 python -u bench.py --mode dense-sim > $M/dense_sim.log 2>&1 || { echo "dense-sim rc=$?"; tail -20 $M/dense_sim.log; exit 1; }
tail -1 $M/dense_sim.log | cut -c1-300
