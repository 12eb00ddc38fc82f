# A/B of wide-tier library variants on the dense executor bench (measurement
# only): bash tools/wide_ab.sh name1 name2 ...  (fantoch_amd/build_<name>/
# libfantoch_amd.so from `make wvariant`; "base" = the in-tree library)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/wab; mkdir -p $M
for v in "$@"; do
  L=""; [ "$v" = base ] || L=fantoch_amd/build_$v/libfantoch_amd.so
  FX_LIB=$L timeout -k 10 200 python3 bench.py --mode dense --no-cpu-baseline > $M/$v.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('%-10s %8.2f M cmds/s  %8.1f ms' % ('$v', d['value']/1e6, d['ms_per_step']))"
done
