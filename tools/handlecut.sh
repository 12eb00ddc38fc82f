# Handle transfers + cut driver: GPU parity tests, then the configs[4] bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/handlecut; rm -rf $M; mkdir -p $M
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_partial.py tests/test_exec_log.py tests/test_golden.py tests/test_cut_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $M/t.log 2>&1 || { echo "pytest rc=$?"; tail -30 $M/t.log; exit 1; }
tail -1 $M/t.log
timeout -k 10 300 python -u bench.py --mode huge --no-cpu-baseline > $M/huge.log 2>&1 || { echo "huge rc=$?"; tail -20 $M/huge.log; exit 1; }
python -c "import json; d=json.loads(open('$M/huge.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
