# round-5: k_simx configs[3] build at 5 waves per SIMD with 2 instances per
# workgroup (build_x5: 20 instances per CU) vs the in-tree 4-wave build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5x5; mkdir -p $M
FX_LIB=fantoch_amd/build_x5/libfantoch_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py tests/test_sim_capture.py tests/test_poison_all.py -k "not pred and not executor and not escalation and not persistent" \
  > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -1 $M/tests.log
run() {  # name seeds env...
  local nm=$1 sd=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 --seeds $sd > $M/$nm.log 2>&1 \
    || { echo "$nm rc=$?"; tail -5 $M/$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$M/$nm.log').read().strip().splitlines()[-1]); print('%-10s %8.2f M cmds/s  %8.1f ms' % ('$nm', d['value']/1e6, d['ms_per_step']))"
}
run w4_4096 4096
run x5_5120 5120 FX_LIB=fantoch_amd/build_x5/libfantoch_amd.so
run x5_4096 4096 FX_LIB=fantoch_amd/build_x5/libfantoch_amd.so
run w4_4096 4096
