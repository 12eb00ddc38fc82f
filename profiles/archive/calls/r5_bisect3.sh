# the intermittent k_simx failure with the invariant checks in: LDS search on, then off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
for cfg in "FX_SIMX_LX=1" "FX_SIMX_LX=0"; do
  env $cfg timeout -k 10 400 python3 -u tools/simx_poison_repeat.py 6 sim_epaxos_5_2,config3_epaxos,sim_atlas_5_2 > $M/rep3_$cfg.log 2>&1
  echo "$cfg rc=$?"; grep -v "done" $M/rep3_$cfg.log | tail -8; tail -1 $M/rep3_$cfg.log
done
