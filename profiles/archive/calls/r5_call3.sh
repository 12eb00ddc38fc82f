# round-5 GPU call 3: the measurement records of the remaining modes and the handle
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PREFIX=gpurun_out/r5prof/r05b_ bash profiles/archive/calls/r5_measure.sh dense huge dense-sim placements || exit 1
PREFIX=gpurun_out/r5prof/r05b_ bash profiles/archive/calls/r5_handle.sh || exit 1
