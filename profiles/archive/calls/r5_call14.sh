# round-5 closing check at HEAD: every GPU test + smoke, the default bench line
# (the driver's command), the k_simx phase split of the 4-wave configs[3] build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash profiles/archive/calls/r5_final_tests.sh || exit 1
M=gpurun_out/r5z; mkdir -p $M
timeout -k 10 600 python3 bench.py > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-200
FX_LIB=fantoch_amd/build_prof6/libfantoch_amd.so timeout -k 10 300 python3 tools/simx_phase.py --seeds 4096 --cmds 50 > $M/phase.log 2>&1 || { echo "phase rc=$?"; tail -5 $M/phase.log; exit 1; }
tail -26 $M/phase.log
