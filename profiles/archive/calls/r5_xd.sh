# round-5: k_simx built with the default scheduler (build_xd) vs the in-tree
# iterative-ILP build, dense-sim at 5,120 instances
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5xd; mkdir -p $M
for v in in xd in xd; do
  L=fantoch_amd/build_$v/libfantoch_amd.so; [ $v = in ] && L=fantoch_amd/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 > $M/$v.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms')"
done
