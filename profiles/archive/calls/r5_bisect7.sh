# which arena table the k_simx failure reads before writing: 256 copies per
# launch over a 0xA5-filled arena, one table group zeroed at a time; then the
# event-log build's first diverging events
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
for mode in fill fill-rec fill-slot fill-ev fill-scr fill-cl; do
  FX_SIMX_ARENA=$mode timeout -k 10 300 python3 -u tools/simx_repro.py --copies 256 --rounds 1 --fills 4:0 \
    --probes sim_epaxos_5_2,config3_epaxos > $M/rep7_$mode.log 2>&1
  echo "arena=$mode rc=$?: $(grep -c odd $M/rep7_$mode.log) lines; $(grep 'odd copies in total' $M/rep7_$mode.log)"
  grep "majority" $M/rep7_$mode.log | sed 's/majority.*x\([0-9]*\);/x\1;/' | cut -c1-160
done
FX_LIB=fantoch_amd/build_evlog/libfantoch_amd.so FX_SIMX_ARENA=fill timeout -k 10 400 python3 -u tools/simx_repro.py \
  --copies 96 --rounds 1 --fills 4:0 --probes sim_epaxos_5_2,config3_epaxos > $M/rep7_evlog.log 2>&1
echo "evlog rc=$?"; tail -40 $M/rep7_evlog.log
