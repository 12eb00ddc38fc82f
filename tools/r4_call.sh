# round-4 GPU call: the k_sim divergence bisection on the iterative-ILP variant,
# then the new GPU tests on the product build
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/poison
FX_LIB=fantoch_amd/build_iilp/libfantoch_amd.so timeout -k 10 300 python -u tools/sim_stale_repro.py --bisect 6120 --probes n7_0 > gpurun_out/poison/bisect.log 2>&1
rc=$?; echo "bisect rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_sim_gpu.py tests/test_partial.py tests/test_sim_large.py -k "basic or partial or both_kernels or info or protocol_sim" > gpurun_out/poison/newtests.log 2>&1
rc=$?; echo "tests rc=$rc"; exit $rc
