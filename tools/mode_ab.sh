# A/B of library variants on any bench mode (measurement only):
# bash tools/mode_ab.sh MODE name1 name2 ...  (fantoch_amd/build_<name>/libfantoch_amd.so
# from make variant / wvariant / fvariant; "base" = the in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
MODE=$1; shift
M=gpurun_out/mab; mkdir -p $M
for v in "$@"; do
  L=""; [ "$v" = base ] || L=fantoch_amd/build_$v/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 300 python3 bench.py --mode $MODE --no-cpu-baseline > $M/$MODE_$v.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $M/$MODE_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$MODE_$v.log').read().strip().splitlines()[-1]); print('%-10s %-10s %8.2f M/s  %8.1f ms' % ('$MODE', '$v', d['value']/1e6, d['ms_per_step']))"
done
