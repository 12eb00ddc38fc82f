# configs[2] sweep at the default dot-table size and at --dot-slots 32
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/plab; rm -rf $M; mkdir -p $M
for ds in ${DSLIST:-0 32}; do
  timeout -k 10 400 python -u bench.py --mode placements --cmds 100 --steps 1 --warmup 0 --no-cpu-baseline --dot-slots $ds > $M/p$ds.log 2>&1 || { echo "p$ds rc=$?"; tail -5 $M/p$ds.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['reruns_at_larger_tables_rank0'], d['all_ok'])" $M/p$ds.log
done
