set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -20 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
PMC_OUT=gpurun_out/pmc_wave_nopend bash tools/pmc.sh --steps 2 --warmup 1 --no-cpu-baseline --window 0 --cycle-pct 0
python tools/pmc_summary.py gpurun_out/pmc_wave_nopend
