# k_simx changes: its parity tests first, then a dense-sim A/B against a
# baseline build (fantoch_amd/build_<base>/) and the in-tree library with and
# without the LDS Tarjan state.  usage: bash profiles/archive/calls/r5_simx.sh [base]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5x; mkdir -p $M
BASE=${1:-xw3}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py tests/test_sim_capture.py tests/test_sim_gpu.py tests/test_poison_all.py tests/test_gpu_parity.py \
  > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -2 $M/tests.log
run() {  # name, env...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 > $M/$nm.log 2>&1 \
    || { echo "$nm rc=$?"; tail -5 $M/$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$M/$nm.log').read().strip().splitlines()[-1]); print('%-8s %8.2f M cmds/s  %8.1f ms' % ('$nm', d['value']/1e6, d['ms_per_step']))"
}
run base FX_LIB=fantoch_amd/build_$BASE/libfantoch_amd.so
run lx FX_SIMX_LX=1
run nolx FX_SIMX_LX=0
