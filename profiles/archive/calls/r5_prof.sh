# k_simx phase split (FX_SIM_PROFILE build) on the dense-sim bench's shape, with and without the LDS Tarjan state
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5p; mkdir -p $M
for lx in 1 0; do
  FX_SIMX_LX=$lx FX_LIB=fantoch_amd/build_prof/libfantoch_amd.so timeout -k 10 300 python3 tools/simx_phase.py --seeds 3072 --cmds 50 \
    --out $M/phase_lx$lx.json > $M/phase_lx$lx.txt 2>&1 || { echo "lx$lx rc=$?"; tail -5 $M/phase_lx$lx.txt; exit 1; }
  echo "== LX=$lx"; cat $M/phase_lx$lx.txt
done
