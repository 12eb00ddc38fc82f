# round-5: the headline k_sim at 5 waves per SIMD with two instances per
# workgroup (build_s5, FX_SIM_WPS5: 20 per CU) vs the in-tree 4-wave build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5s5; mkdir -p $M
FX_LIB=fantoch_amd/build_s5/libfantoch_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_sim_gpu.py tests/test_sim_poison.py > $M/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $M/tests.log; exit 1; }
tail -1 $M/tests.log
for v in in s5 in s5; do
  L=fantoch_amd/build_$v/libfantoch_amd.so; [ $v = in ] && L=fantoch_amd/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline > $M/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms')"
done
