# k_simx A/B: the in-tree build (3 waves per SIMD; with / without the row
# prefetch) vs build_lxw4 (4 waves per SIMD), dense-sim at 3,072 and 4,096 instances
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5o; mkdir -p $M
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py tests/test_sim_capture.py > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -1 $M/tests.log
run() {  # name seeds env...
  local nm=$1 sd=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 --seeds $sd > $M/$nm.log 2>&1 \
    || { echo "$nm rc=$?"; tail -5 $M/$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$M/$nm.log').read().strip().splitlines()[-1]); print('%-10s %8.2f M cmds/s  %8.1f ms' % ('$nm', d['value']/1e6, d['ms_per_step']))"
}
run w3 3072
run w3_nopf 3072 FX_SIMX_PF=0
run w3_4096 4096
run w4_3072 3072 FX_LIB=fantoch_amd/build_lxw4/libfantoch_amd.so
run w4_4096 4096 FX_LIB=fantoch_amd/build_lxw4/libfantoch_amd.so
