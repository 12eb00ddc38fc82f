# A/B of wide-tier library variants on the dense executor bench (measurement only):
# bash tools/dense_ab.sh name1 name2 ...  (fantoch_amd/build_<name>/libfantoch_amd.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  FX_LIB=fantoch_amd/build_$v/libfantoch_amd.so timeout -k 10 300 python bench.py --mode dense --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dab.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/dab.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/dab.log').read().strip().splitlines()[-1]); print(sys.argv[1], '%.2f M' % (d['value']/1e6), d['ms_per_step'])" $v
done
