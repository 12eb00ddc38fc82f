# round-5: k_simx's configs[3] build at 4 waves per SIMD (dense-sim at 4,096
# instances): its GPU tests (poisoned too) and the dense-sim record; then the
# k_pred two-streams-per-workgroup build: its tests and record
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5w; mkdir -p $M
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py tests/test_sim_capture.py tests/test_poison_all.py tests/test_pred_gpu.py > $M/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -1 $M/tests.log
PREFIX=gpurun_out/r5prof/r05h_ bash profiles/archive/calls/r5_measure.sh dense-sim pred || exit 1
