# round-5 call: the GPU tests (profiles/archive/calls/r5_tests.sh), then the k_simx occupancy A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/archive/calls/r5_tests.sh || exit 1
M=gpurun_out/xab; mkdir -p $M
for v in xw3 xw4; do
  for s in 3072 4096; do
    FX_LIB=fantoch_amd/build_$v/libfantoch_amd.so timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 --seeds $s > $M/${v}_$s.log 2>&1 \
      || { echo "$v rc=$?"; tail -5 $M/${v}_$s.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$M/${v}_$s.log').read().strip().splitlines()[-1]); print('%-6s %5d %8.2f M cmds/s  %8.1f ms' % ('$v', $s, d['value']/1e6, d['ms_per_step']))"
  done
done
