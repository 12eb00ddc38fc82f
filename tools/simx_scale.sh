# dense-sim throughput against the number of instances in flight (k_simx's
# arena working set vs the caches).  usage: bash tools/simx_scale.sh "768 1536 3072"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sx
for s in $1; do
  timeout -k 10 300 python3 bench.py --mode dense-sim --seeds $s --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sx/$s.log 2>&1 || { echo "rc=$? at $s"; tail -5 gpurun_out/sx/$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms')" gpurun_out/sx/$s.log $s
done
