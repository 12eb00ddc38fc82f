set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/simcheck; rm -rf $M; mkdir -p $M
timeout -k 10 400 python -u -m pytest tests/test_sim_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $M/t.log 2>&1 || { echo "pytest rc=$?"; tail -30 $M/t.log; exit 1; }
tail -2 $M/t.log
if [ -n "$PHASE" ]; then
FX_LIB=fantoch_amd/build_prof/libfantoch_amd.so timeout -k 10 200 python tools/sim_phase.py --seeds 256 --cmds 1000 > $M/phase.log 2>&1 || { echo phase failed; tail $M/phase.log; exit 1; }
cat $M/phase.log
fi
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-400
