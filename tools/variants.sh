set -e
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
$B > gpurun_out/v_default.log 2>&1
$B --window 0 --cycle-pct 0 > gpurun_out/v_nopend.log 2>&1
$B --conflicts 0 > gpurun_out/v_c0.log 2>&1
$B --conflicts 100 > gpurun_out/v_c100.log 2>&1
$B --conflicts 0 --window 0 --cycle-pct 0 > gpurun_out/v_c0_w0.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
