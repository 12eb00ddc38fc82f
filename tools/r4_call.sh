# round-4 GPU call: the zero-fill poisoned test against the pre-fix
# iterative-ILP k_sim (must fail: the test catches the round-3 defect), then an
# A/B of the fixed k_sim builds (default vs iterative-ILP schedule) on configs[1]
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/poison
FX_LIB=fantoch_amd/build_iilp_old/libfantoch_amd.so timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_sim_poison.py -k "n7 or no_gc" > gpurun_out/poison/old_iilp_poison.log 2>&1
rc=$?; echo "old iilp poison rc=$rc (1 expected)"; if [ $rc -ne 1 ] && [ $rc -ne 0 ]; then exit $rc; fi
bash tools/sim_ab.sh base iilp base iilp
