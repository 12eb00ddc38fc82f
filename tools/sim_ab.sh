# A/B of k_sim library variants on the configs[1] bench (measurement only):
# bash tools/sim_ab.sh name1 name2 ...  (fantoch_amd/build_<name>/libfantoch_amd.so,
# "base" = the in-tree library, "generic" = the in-tree library with --generic)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/ab; mkdir -p $M
for v in "$@"; do
  X=""; L=""
  case $v in
    base) ;;
    generic) X="--generic" ;;
    *) L=fantoch_amd/build_$v/libfantoch_amd.so ;;
  esac
  FX_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $X > $M/$v.log 2>&1 \
    || { echo "$v rc=$?"; tail -5 $M/$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$M/$v.log').read().strip().splitlines()[-1]); print('%-10s %8.1f M cmds/s  %8.1f ms  reruns %s' % ('$v', d['value']/1e6, d['ms_per_step'], d.get('reruns_at_larger_tables_rank0')))"
done
