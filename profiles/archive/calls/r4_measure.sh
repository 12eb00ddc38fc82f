# round-4 measurement: GPU tests + smoke, then for each secondary bench mode the
# counter passes of its dominant kernel (tools/mode_pmc.sh) summarised into
# profiles/pmc_<mode>.json, then the bench lines that read them
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r4m; mkdir -p $M
P=${PREFIX:-profiles/r04a_}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $M/gputest.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -2 $M/gputest.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
for spec in "dense-sim k_simx" "dense k_graph_wide<false>" "pred k_pred<false>" "placements k_sim<"; do
  set -- $spec; mode=$1; pat=$2
  extra=""; [ $mode = placements ] && extra="--cmds 100"
  bash tools/mode_pmc.sh $mode "$pat" $extra || exit 1
  python3 tools/mode_pmc_summary.py $mode gpurun_out/pmc_$mode "$pat" $P $extra > $M/${mode}_summary.log 2>&1 || { echo "summary $mode failed"; tail -5 $M/${mode}_summary.log; exit 1; }
  cp gpurun_out/pmc_$mode/trace/*kernel_stats.csv ${P}${mode}_kernel_stats.csv 2>/dev/null
  timeout -k 10 600 python3 bench.py --mode $mode $extra > $M/$mode.log 2>&1 || { echo "bench $mode rc=$?"; tail -5 $M/$mode.log; exit 1; }
  tail -1 $M/$mode.log > ${P}${mode}_bench.json
  echo "$mode: $(python3 -c "import json;d=json.load(open('${P}${mode}_bench.json'));r=d.get('roofline') or {};print(round(d['value']/1e6,1),'M', 'frac',r.get('frac'),'traffic',r.get('traffic'),'t/alg',r.get('traffic_over_alg'),'waves',(r.get('issue') or {}).get('mean_waves_per_cu'))")"
done
