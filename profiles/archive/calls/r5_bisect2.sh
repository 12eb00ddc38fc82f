# the intermittent poisoned configs[3] failure: round-4 build vs the switches of the new one
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
for cfg in "FX_LIB=fantoch_amd/build_xw3/libfantoch_amd.so" "FX_SIMX_LX=0" "FX_SIMX_PF=0" "FX_SIMX_PF=1"; do
  nm=$(echo $cfg | tr '=/' '__')
  env $cfg timeout -k 10 300 python3 -u tools/simx_poison_repeat.py 5 > $M/rep_$nm.log 2>&1
  echo "$cfg rc=$?"; grep -v "done" $M/rep_$nm.log | tail -6; tail -1 $M/rep_$nm.log
done
