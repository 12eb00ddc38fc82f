# configs[1] simulator step time per conflict rate (4096 instances each) and in
# both launch orders of the full sweep.  usage: bash tools/sim_rates.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rates
for c in 0 2 10 50 100 "100,50,10,2,0" "0,2,10,50,100"; do
  timeout -k 10 300 python3 bench.py --conflicts $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rates/r.log 2>&1 || { echo "rc=$? at $c"; tail -5 gpurun_out/rates/r.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms')" gpurun_out/rates/r.log "$c"
done
