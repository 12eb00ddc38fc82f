# GPU tests, then the split tier's default bench and threshold sweep.
# usage: bash tools/split_eval.sh "8 12 16 24"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gputest.log 2>&1
rc=$?
tail -3 gpurun_out/gputest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
for thr in $1; do
  FX_SPLIT_THRESHOLD=$thr timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline > gpurun_out/split_$thr.log 2>&1 || { echo "thr $thr rc=$?"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('thr', sys.argv[2], '%.3f G' % (d['value']/1e9), d['roofline']['kernel_ms_avg'])" gpurun_out/split_$thr.log $thr
done
