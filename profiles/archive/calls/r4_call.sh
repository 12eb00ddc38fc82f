set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r4/ptest.log 2>&1
rc=$?; tail -3 gpurun_out/r4/ptest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode handle > gpurun_out/r4/handle.log 2>&1
rc=$?; echo "bench handle rc=$rc"; python3 -c "import json;d=json.loads(open('gpurun_out/r4/handle.log').read().strip().splitlines()[-1]);print('py',d['gpu_us_per_add'],'cpp',d['gpu_us_per_add_cpp_loop'],d['gpu_cpp_loop'],'parity',d['order_parity'])"; exit $rc
