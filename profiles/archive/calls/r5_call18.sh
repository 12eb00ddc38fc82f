# round-5 closing check 3 at HEAD: every GPU test + smoke, the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/archive/calls/r5_final_tests.sh || exit 1
M=gpurun_out/r5z; mkdir -p $M
timeout -k 10 600 python3 bench.py > $M/bench3.log 2>&1 || { echo "bench rc=$?"; tail -5 $M/bench3.log; exit 1; }
tail -1 $M/bench3.log | cut -c1-200
