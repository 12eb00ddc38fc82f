# round-5 GPU call 11: configs[3] at the reference's C4 sizing (1,000 commands
# per client) with the bench's 3,072 instances, one step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5c4; mkdir -p $M
timeout -k 10 900 python3 -u bench.py --mode dense-sim --cmds 1000 --steps 1 --warmup 0 \
  --cpu-baseline-seconds 20 > $M/bench3072.log 2>&1 || { echo "c4 rc=$?"; tail -5 $M/bench3072.log; exit 1; }
tail -1 $M/bench3072.log | cut -c1-300
