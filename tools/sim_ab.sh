set -e
cd "$GRAFT_REPO_ROOT"
for c in ${CMDS:-1000 200}; do
  FX_LIB=${OLD_LIB:-fantoch_amd/build_old/libfantoch_amd.so} timeout -k 10 300 python bench.py --steps 2 --cmds $c --no-cpu-baseline > gpurun_out/ab_old_$c.log 2>&1
  timeout -k 10 300 python bench.py --steps 2 --cmds $c --no-cpu-baseline > gpurun_out/ab_new_$c.log 2>&1
done
for f in gpurun_out/ab_*.log; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms', d['executed_per_step'], d['roofline']['traffic'])" $f; done
