# the intermittent k_simx failure with the invariant checks (event tree, SCC members) in the shipped build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
timeout -k 10 800 python3 -u tools/simx_poison_repeat.py 14 sim_epaxos_5_2,config3_epaxos,sim_atlas_5_2 > $M/rep5.log 2>&1
echo "rc=$?"; grep -v "done" $M/rep5.log | tail -10; tail -1 $M/rep5.log
