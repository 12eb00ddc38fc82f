# round-5 GPU call 5: k_pred's compiled-in SMALL layout: its GPU tests (poisoned too), measurement record
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5p; mkdir -p $M
timeout -k 10 400 python -u -m pytest tests/test_pred_gpu.py tests/test_poison_all.py -k "pred" -x -q --timeout 200 \
  --timeout-method thread > $M/tests6.log 2>&1 || { echo "pred tests rc=$?"; tail -30 $M/tests6.log; exit 1; }
tail -1 $M/tests6.log
PREFIX=gpurun_out/r5prof/r05e_ bash profiles/archive/calls/r5_measure.sh pred || exit 1
