# k_simx: parity tests, the dense-sim bench vs a baseline build, and the phase split (FX_SIM_PROFILE build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5y; mkdir -p $M
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_large.py tests/test_sim_capture.py tests/test_poison_all.py -k "simx or config3 or reference or capture or small or extra or capacity or arena" \
  > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -1 $M/tests.log
run() {  # name env...
  local nm=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 > $M/$nm.log 2>&1 \
    || { echo "$nm rc=$?"; tail -5 $M/$nm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$M/$nm.log').read().strip().splitlines()[-1]); print('%-10s %8.2f M cmds/s  %8.1f ms' % ('$nm', d['value']/1e6, d['ms_per_step']))"
}
run base FX_LIB=fantoch_amd/build_${1:-xw3}/libfantoch_amd.so
run new
FX_LIB=fantoch_amd/build_prof/libfantoch_amd.so timeout -k 10 300 python3 tools/simx_phase.py --seeds 3072 --cmds 50 \
  --out $M/phase.json > $M/phase.txt 2>&1 || { echo "phase rc=$?"; tail -5 $M/phase.txt; exit 1; }
cat $M/phase.txt
