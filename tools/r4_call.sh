set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
bash tools/sim_ab.sh base gcu base gcu || exit 1
FX_LIB=fantoch_amd/build_gcu/libfantoch_amd.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_sim_gpu.py tests/test_sim_poison.py > gpurun_out/r4/gcu_tests.log 2>&1
rc=$?; echo "gcu tests rc=$rc"; tail -2 gpurun_out/r4/gcu_tests.log; exit $rc
