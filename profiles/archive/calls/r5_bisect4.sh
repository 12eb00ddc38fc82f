# the intermittent k_simx failure: does the round-4 build (build_xw3) show it too?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
FX_LIB=fantoch_amd/build_xw3/libfantoch_amd.so timeout -k 10 700 python3 -u tools/simx_poison_repeat.py 12 sim_epaxos_5_2,config3_epaxos,sim_atlas_5_2 > $M/rep4_xw3.log 2>&1
echo "xw3 rc=$?"; grep -v "done" $M/rep4_xw3.log | tail -8; tail -1 $M/rep4_xw3.log
