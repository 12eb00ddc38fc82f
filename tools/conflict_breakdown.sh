# Step time of the default split tier on subsets of BASELINE configs[1]:
# usage: bash tools/conflict_breakdown.sh "100:4096 100:2048 50:4096 ..."  (conflicts:seeds)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/diag
for cs in $1; do
  c=${cs%%:*}; s=${cs##*:}
  timeout -k 10 200 python bench.py --mode executor --steps 3 --no-cpu-baseline --conflicts $c --seeds $s $2 > gpurun_out/diag/c.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/diag/c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.3f G' % (d['value']/1e9), d['ms_per_step'], d['roofline']['kernel_ms_avg'])" gpurun_out/diag/c.log "$cs"
done
