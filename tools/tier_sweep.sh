# per-tier executor throughput on the default bench and its conflict extremes
# usage: bash tools/tier_sweep.sh "0 3 1" ; outputs gpurun_out/t_<tier>_<variant>.log
mkdir -p gpurun_out
for t in $1; do
  for v in "default:" "c0:--conflicts 0" "c100:--conflicts 100" "nopend:--window 0 --cycle-pct 0"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --tier $t $args > gpurun_out/t_${t}_$name.log 2>&1 || { echo "tier $t $name rc=$?"; tail -3 gpurun_out/t_${t}_$name.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.3f G' % (d['value']/1e9), d['roofline']['kernel_ms_avg'])" gpurun_out/t_${t}_$name.log $t $name
  done
done
