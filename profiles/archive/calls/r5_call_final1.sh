# round-5 GPU call: every GPU test + smoke, then the measurement records of
# the headline, executor, huge and handle modes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/archive/calls/r5_final_tests.sh || exit 1
PREFIX=gpurun_out/r5prof/r05a_ bash profiles/archive/calls/r5_measure.sh sim executor huge || exit 1
PREFIX=gpurun_out/r5prof/r05a_ bash profiles/archive/calls/r5_handle.sh || exit 1
