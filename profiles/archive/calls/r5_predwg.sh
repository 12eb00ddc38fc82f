# round-5: k_pred streams per workgroup A/B (compiled n = 5 SMALL build): 1, 2
# (in-tree), 4; the 4-stream build's pred GPU tests first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5pw; mkdir -p $M
FX_LIB=fantoch_amd/build_pw4/libfantoch_amd.so timeout -k 10 300 python -u -m pytest tests/test_pred_gpu.py -x -q --timeout 200 \
  --timeout-method thread > $M/tests4.log 2>&1 || { echo "tests rc=$?"; tail -30 $M/tests4.log; exit 1; }
tail -1 $M/tests4.log
for v in pw1 in pw4 in; do
  L=fantoch_amd/build_$v/libfantoch_amd.so; [ $v = in ] && L=fantoch_amd/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 300 python3 bench.py --mode pred --no-cpu-baseline > $M/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms reruns', d['reruns'])"
done
