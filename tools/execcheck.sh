# Executor parity + step times after an executor-kernel change:
# GPU parity tests, the 100 % conflict subset on tier 0 and on the default
# split tier, and the whole executor bench.  Stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/execcheck; rm -rf $M; mkdir -p $M
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_cut_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $M/t.log 2>&1 || { echo "pytest rc=$?"; tail -30 $M/t.log; exit 1; }
tail -2 $M/t.log
bash tools/conflict_breakdown.sh "100:4096" "--tier 0" || exit 1
bash tools/conflict_breakdown.sh "100:4096" || exit 1
timeout -k 10 300 python -u bench.py --mode executor --steps 3 --no-cpu-baseline > $M/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $M/bench.log; exit 1; }
tail -1 $M/bench.log | cut -c1-300
python -c "import json; d=json.loads(open('$M/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])"
