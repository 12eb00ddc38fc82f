# Round 5: new GPU tests first (-x stops at the first failure), then the whole
# GPU suite, smoke and the headline bench line (histogram parity on its sample).
# usage: bash profiles/archive/calls/r5_tests.sh [pytest selection for the first step]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5; mkdir -p $M
FIRST=${1:-"tests/test_poison_all.py tests/test_gpu_parity.py"}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $FIRST \
  > $M/first.log 2>&1 || { echo "first rc=$?"; tail -30 $M/first.log; exit 1; }
tail -2 $M/first.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > $M/gputest.log 2>&1 || { echo "gputest rc=$?"; tail -30 $M/gputest.log; exit 1; }
tail -2 $M/gputest.log
timeout -k 10 240 python -u __graft_entry__.py smoke > $M/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $M/smoke.log; exit 1; }
tail -2 $M/smoke.log
timeout -k 10 400 python -u bench.py > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-400
