# round-5: the LDS search of k_simx (FX_SIMX_LX=1) under register poisoning on
# the zeroed arena, its parity tests, then the dense-sim bench line with it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5lx; mkdir -p $M
FX_SIMX_LX=1 timeout -k 10 420 python3 -u tools/simx_poison_repeat.py 6 > $M/poison.log 2>&1 \
  || { echo "poison rc=$?"; tail -20 $M/poison.log; exit 1; }
tail -2 $M/poison.log
FX_SIMX_LX=1 timeout -k 10 400 python -u -m pytest tests/test_sim_large.py tests/test_poison_all.py -k "simx or sim_large or config3 or reference" \
  -x -q --timeout 300 --timeout-method thread > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $M/tests.log; exit 1; }
tail -1 $M/tests.log
FX_SIMX_LX=1 timeout -k 10 400 python3 bench.py --mode dense-sim > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-200
