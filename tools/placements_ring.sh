# configs[2] sweep at several message-pool sizes (RINGLIST), default dot tables
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/plring; rm -rf $M; mkdir -p $M
for r in ${RINGLIST:-0 160}; do
  timeout -k 10 400 python -u bench.py --mode placements --cmds 100 --steps 1 --warmup 0 --no-cpu-baseline --ring-entries $r > $M/r$r.log 2>&1 || { echo "r$r rc=$?"; tail -5 $M/r$r.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['reruns_at_larger_tables_rank0'], d['all_ok'])" $M/r$r.log
done
