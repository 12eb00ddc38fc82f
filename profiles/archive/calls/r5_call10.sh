# round-5 GPU call 10: every GPU test + smoke at HEAD, the dense-sim record
# (compiled configs[3] geometry), and configs[3] at the reference's C4 sizing
# (1,000 commands per client: the pending set of a long run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/archive/calls/r5_final_tests.sh || exit 1
PREFIX=gpurun_out/r5prof/r05f_ bash profiles/archive/calls/r5_measure.sh dense-sim || exit 1
M=gpurun_out/r5c4; mkdir -p $M
timeout -k 10 900 python3 bench.py --mode dense-sim --cmds 1000 --seeds 384 --steps 1 --warmup 0 \
  --cpu-baseline-seconds 20 > $M/bench.log 2>&1 || { echo "c4 rc=$?"; tail -5 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-300
