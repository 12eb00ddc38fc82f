set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python -u bench.py --cmds 200 --steps 2 --no-cpu-baseline > gpurun_out/b3.log 2>&1 || exit 1
FX_LIB=fantoch_amd/build_w4/libfantoch_amd.so timeout -k 10 300 python -u bench.py --cmds 200 --steps 2 --no-cpu-baseline > gpurun_out/b4.log 2>&1 || exit 1
for f in b3 b4; do python3 -c "import json; j=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', j['value'], j['ms_per_step'])"; done
