# the intermittent k_simx failure vs the arena's initial contents and caching
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
for mode in fill zero uc; do
  FX_SIMX_ARENA=$mode timeout -k 10 400 python3 -u tools/simx_poison_repeat.py 8 sim_epaxos_5_2,config3_epaxos,sim_atlas_5_2 > $M/rep6_$mode.log 2>&1
  echo "arena=$mode rc=$?"; grep -v "done" $M/rep6_$mode.log | tail -8; tail -1 $M/rep6_$mode.log
done
