# round-4 GPU call: the persistent handle (tests, then bench --mode handle),
# then the whole measurement (tools/r4_measure.sh)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "executor" > gpurun_out/r4/handle_tests.log 2>&1
rc=$?; echo "handle tests rc=$rc"; tail -3 gpurun_out/r4/handle_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --mode handle > gpurun_out/r4/handle.log 2>&1
rc=$?; echo "bench handle rc=$rc"; tail -c 600 gpurun_out/r4/handle.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/r4_measure.sh
