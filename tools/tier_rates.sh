# executor time per conflict-rate subset and tier (kernel ms from HIP events)
# usage: bash tools/tier_rates.sh "0 5" "0,2,10 50,100 50 100"
for t in $1; do
  for c in $2; do
    timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --tier $t --conflicts $c > gpurun_out/r_${t}_$c.log 2>&1 || { echo "tier $t $c rc=$?"; tail -3 gpurun_out/r_${t}_$c.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('tier', sys.argv[2], 'rates', sys.argv[3], '%.3f G' % (d['value']/1e9), d['roofline']['kernel_ms_avg'])" gpurun_out/r_${t}_$c.log $t $c
  done
done
