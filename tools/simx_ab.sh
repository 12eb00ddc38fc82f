# A/B of k_simx library variants on the dense-sim bench (measurement only):
# bash tools/simx_ab.sh name1 name2 ...  (fantoch_amd/build_<name>/libfantoch_amd.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/xab; mkdir -p $M
for v in "$@"; do
  FX_LIB=fantoch_amd/build_$v/libfantoch_amd.so timeout -k 10 300 python3 bench.py --mode dense-sim --no-cpu-baseline --steps 2 --warmup 1 > $M/$v.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('%-10s %8.2f M cmds/s  %8.1f ms' % ('$v', d['value']/1e6, d['ms_per_step']))"
done
