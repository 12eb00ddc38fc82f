# k_sim schedule-dependence diagnostics (round 4): the iterative-ILP variant
# (make variant V=iilp D="-mllvm -amdgpu-sched-strategy=iterative-ilp") and the
# default build on tools/sim_stale_repro.py
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/poison
FX_LIB=fantoch_amd/build_iilp/libfantoch_amd.so timeout -k 10 300 python -u tools/sim_stale_repro.py $@ > gpurun_out/poison/repro_iilp.log 2>&1
rc=$?; echo "iilp rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/sim_stale_repro.py $@ > gpurun_out/poison/repro_def.log 2>&1
rc=$?; echo "def rc=$rc"
exit $rc
