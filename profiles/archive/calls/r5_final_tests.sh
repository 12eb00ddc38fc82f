# round-5 closing checks: every GPU test, smoke (outputs under gpurun_out/r5f/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5f; mkdir -p $M
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $M/gputest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $M/gputest.log; exit 1; }
tail -2 $M/gputest.log
timeout -k 10 240 python -u __graft_entry__.py smoke > $M/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $M/smoke.log; exit 1; }
tail -2 $M/smoke.log
