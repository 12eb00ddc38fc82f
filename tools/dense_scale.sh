# dense executor (configs[3] streams) throughput against the instances per launch.
# usage: bash tools/dense_scale.sh "768 1536"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ds
for s in $1; do
  timeout -k 10 400 python3 bench.py --mode dense --seeds $s --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ds/$s.log 2>&1 || { echo "rc=$? at $s"; tail -5 gpurun_out/ds/$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms', d['roofline'].get('kernel_ms_avg'))" gpurun_out/ds/$s.log $s
done
