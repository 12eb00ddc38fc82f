# Persistent handles and hardware queues: the same Add stream through H handles
# driven from one thread, per stream kind (FX_PERSIST_QUEUE).  Each run under
# its own time limit; a run that stalls on a shared queue shows as rc=124.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/qp
BENCH_HANDLE_KEEP_STREAM=gpurun_out/qp/stream.bin timeout -k 10 300 python -u bench.py --mode handle > gpurun_out/qp/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/qp/bench.log; exit 1; }
for q in cumask prio plain; do
  for h in 1 6; do
    FX_PERSIST_QUEUE=$q timeout -k 5 40 tools/build/handle_latency gpurun_out/qp/stream.bin 2 $h > gpurun_out/qp/$q.$h.log 2>&1
    rc=$?
    echo "$q H=$h rc=$rc $(grep -o '"handles.*us_per_add_min": [0-9.]*' gpurun_out/qp/$q.$h.log)"
    [ $rc -eq 0 ] || [ $rc -eq 124 ] || exit 1
  done
done
