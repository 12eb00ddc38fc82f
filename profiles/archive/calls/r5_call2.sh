# round-5 GPU call 2: every GPU test + smoke (the XCD-aware stream mapping of
# k_pred / k_graph_wide and the pred row prefetch), then the measurement
# records of the remaining modes and the handle
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/archive/calls/r5_final_tests.sh || exit 1
PREFIX=gpurun_out/r5prof/r05b_ bash profiles/archive/calls/r5_measure.sh pred dense huge dense-sim placements || exit 1
PREFIX=gpurun_out/r5prof/r05b_ bash profiles/archive/calls/r5_handle.sh || exit 1
