# configs[3] dense path: wide-tier parity tests, then the dense bench (no CPU baseline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/densecheck; rm -rf $M; mkdir -p $M
timeout -k 10 500 python -u -m pytest tests/test_wide_gpu.py tests/test_sim_capture.py tests/test_partial.py -m gpu -x -q --timeout 300 --timeout-method thread > $M/t.log 2>&1 || { echo "pytest rc=$?"; tail -30 $M/t.log; exit 1; }
tail -2 $M/t.log
timeout -k 10 300 python -u bench.py --mode dense --no-cpu-baseline "$@" > $M/dense.log 2>&1 || { echo "dense rc=$?"; tail -20 $M/dense.log; exit 1; }
python -c "import json; d=json.loads(open('$M/dense.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['tier_counts'], d['chain_size_max'])"
