# round-5 GPU call 4: the lane-parallel phase checks of k_pred (its GPU tests,
# poisoned too, and its measurement record), then the LDS search of k_simx
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5p; mkdir -p $M
timeout -k 10 400 python -u -m pytest tests/test_pred_gpu.py tests/test_poison_all.py -k "pred" -x -q --timeout 200 \
  --timeout-method thread > $M/tests.log 2>&1 || { echo "pred tests rc=$?"; tail -30 $M/tests.log; exit 1; }
tail -1 $M/tests.log
PREFIX=gpurun_out/r5prof/r05c_ bash profiles/archive/calls/r5_measure.sh pred || exit 1
bash profiles/archive/calls/r5_lx.sh || exit 1
