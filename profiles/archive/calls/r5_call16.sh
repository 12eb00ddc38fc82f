# round-5: k_simx's configs[3] build at 5 waves per SIMD, 2 instances per
# workgroup (in-tree): its GPU tests, the dense-sim record at 5,120 instances;
# then a 6-wave A/B (build_x6) at 6,144
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5x6; mkdir -p $M
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py tests/test_sim_capture.py tests/test_poison_all.py -k "not pred and not executor and not escalation and not persistent" \
  > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -1 $M/tests.log
PREFIX=gpurun_out/r5prof/r05k_ bash profiles/archive/calls/r5_measure.sh dense-sim || exit 1
FX_LIB=fantoch_amd/build_x6/libfantoch_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py -k config3 > $M/tests6.log 2>&1 || { echo "tests6 rc=$?"; tail -40 $M/tests6.log; exit 1; }
tail -1 $M/tests6.log
for v in x6_6144 in_5120; do
  L=fantoch_amd/build_x6/libfantoch_amd.so; sd=6144; [ $v = in_5120 ] && { L=fantoch_amd/libfantoch_amd.so; sd=5120; }
  FX_LIB=$L timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 --seeds $sd > $M/$v.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms')"
done
