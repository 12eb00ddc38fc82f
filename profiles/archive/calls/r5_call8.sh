# round-5 GPU call 8: k_simx reading rare arguments and spec fields on demand: its GPU
# tests (poisoned too), then dense-sim with and without it on the same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5h; mkdir -p $M
timeout -k 10 600 python -u -m pytest tests/test_sim_large.py tests/test_poison_all.py tests/test_sim_capture.py -k "not pred and not executor and not escalation and not persistent" \
  -x -q --timeout 300 --timeout-method thread > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $M/tests.log; exit 1; }
tail -1 $M/tests.log
for gs in 1 0; do
  FX_SIMX_GS=$gs timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline > $M/bench_gs$gs.log 2>&1 || { echo "bench rc=$?"; tail -5 $M/bench_gs$gs.log; exit 1; }
  echo "GS=$gs $(tail -1 $M/bench_gs$gs.log | cut -c1-120)"
done
