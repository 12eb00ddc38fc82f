# round-5: the wide tier (dense executor) with 1 (in-tree), 2 and 5 streams
# per workgroup; the wide GPU tests of each variant first, then dense A/B
# (the CPU sample parity on for every line)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5ww; mkdir -p $M
for v in ww2 ww5; do
  FX_LIB=fantoch_amd/build_$v/libfantoch_amd.so timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py -x -q --timeout 200 \
    --timeout-method thread > $M/tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -30 $M/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $M/tests_$v.log)"
done
for v in in ww2 ww5 in ww5; do
  L=fantoch_amd/build_$v/libfantoch_amd.so; [ $v = in ] && L=fantoch_amd/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 400 python3 bench.py --mode dense > $M/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms parity', d['cpu_baseline'].get('sample_parity'), 'tiers', d.get('tier_counts'))"
done
