# round-5 GPU call 9: k_simx LX A/B on one box (the LDS Tarjan state, opt-in)
# and the phase split of the current build (FX_SIM_PROFILE variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5i; mkdir -p $M
for lx in 0 1 0 1; do
  FX_SIMX_LX=$lx timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline > $M/bench_lx$lx.log 2>&1 || { echo "bench rc=$?"; tail -5 $M/bench_lx$lx.log; exit 1; }
  echo "LX=$lx $(tail -1 $M/bench_lx$lx.log | cut -c90-140)"
done
FX_LIB=fantoch_amd/build_prof5/libfantoch_amd.so timeout -k 10 300 python3 tools/simx_phase.py > $M/phase.log 2>&1 || { echo "phase rc=$?"; tail -5 $M/phase.log; exit 1; }
cat $M/phase.log | tail -30
