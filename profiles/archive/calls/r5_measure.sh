# round-5 measurement records: for each bench mode given (default: all), the
# counter passes of its dominant kernel (tools/mode_pmc.sh) summarised into
# profiles/pmc_<mode>.json, the rocprofv3 kernel stats, then the bench line
# that attaches them (<prefix><mode>_bench.json).  Everything lands under
# gpurun_out/r5prof/ (gpurun brings that directory back; copy the files into
# profiles/ afterwards).  Stops at the first failing step.
# usage: PREFIX=gpurun_out/r5prof/r05a_ bash profiles/archive/calls/r5_measure.sh [mode ...]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5m; mkdir -p $M
P=${PREFIX:-gpurun_out/r5prof/r05a_}
mkdir -p $(dirname $P)
MODES=${*:-"sim dense-sim executor huge dense pred placements"}
for mode in $MODES; do
  extra=""
  case $mode in
    sim) pat="k_sim<" ;;
    dense-sim) pat="k_simx" ;;
    executor) pat="k_graph_lane" ;;
    huge) pat="sum:fx::!k_synth:2" ;;
    dense) pat="k_graph_wide<false" ;;
    pred) pat="k_pred<false" ;;
    placements) pat="k_sim<"; extra="--cmds 100" ;;
    *) echo "unknown mode $mode"; exit 1 ;;
  esac
  bash tools/mode_pmc.sh $mode "$pat" $extra || exit 1
  python3 tools/mode_pmc_summary.py $mode gpurun_out/pmc_$mode "$pat" $P $extra > $M/${mode}_summary.log 2>&1 \
    || { echo "summary $mode failed"; tail -5 $M/${mode}_summary.log; exit 1; }
  cp gpurun_out/pmc_$mode/trace/*kernel_stats.csv ${P}${mode}_kernel_stats.csv 2>/dev/null
  cp profiles/pmc_$mode.json $(dirname $P)/ 2>/dev/null
  timeout -k 10 600 python3 bench.py --mode $mode $extra > $M/$mode.log 2>&1 || { echo "bench $mode rc=$?"; tail -5 $M/$mode.log; exit 1; }
  tail -1 $M/$mode.log > ${P}${mode}_bench.json
  echo "$mode: $(python3 -c "import json;d=json.load(open('${P}${mode}_bench.json'));r=d.get('roofline') or {};c=d.get('cpu_baseline') or {};print(round(d['value']/1e6,2),'M', 'frac',r.get('frac'),'traffic',r.get('traffic'),'t/alg',r.get('traffic_over_alg'),'parity',c.get('sample_parity'))")"
done
