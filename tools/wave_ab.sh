cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in wbase wcanon wbase wcanon; do
  FX_LIB=fantoch_amd/build_$v/libfantoch_amd.so timeout -k 10 200 python bench.py --mode executor --steps 3 --no-cpu-baseline --conflicts 100 --seeds 4096 --tier 4 > gpurun_out/wab.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/wab.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/wab.log').read().strip().splitlines()[-1]); print(sys.argv[1], '%.3f G' % (d['value']/1e9), d['ms_per_step'])" $v
done
