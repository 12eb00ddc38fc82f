# round-5: k_pred 6.7 KB tables (in-tree) vs 32 index slots per source and
# 256-bit windows (build_pw4t: 5.6 KB, 28 streams per CU); the GPU
# pred tests of both first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5pw3; mkdir -p $M
for v in in pw4t; do
  L=fantoch_amd/build_$v/libfantoch_amd.so; [ $v = in ] && L=fantoch_amd/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_pred_gpu.py tests/test_poison_all.py -k pred -x -q --timeout 200 \
    --timeout-method thread > $M/tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -30 $M/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $M/tests_$v.log)"
done
for v in in pw4t in pw4t; do
  L=fantoch_amd/build_$v/libfantoch_amd.so; [ $v = in ] && L=fantoch_amd/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 300 python3 bench.py --mode pred --no-cpu-baseline > $M/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms reruns', d['reruns'])"
done
