# round-5: k_pred 4 streams per workgroup, 5.6 KB compiled tables: its GPU tests (poisoned too), measurement record
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5p; mkdir -p $M
timeout -k 10 400 python -u -m pytest tests/test_pred_gpu.py tests/test_poison_all.py -k "pred" -x -q --timeout 200 \
  --timeout-method thread > $M/tests8.log 2>&1 || { echo "pred tests rc=$?"; tail -30 $M/tests8.log; exit 1; }
tail -1 $M/tests8.log
PREFIX=gpurun_out/r5prof/r05j_ bash profiles/archive/calls/r5_measure.sh pred || exit 1
