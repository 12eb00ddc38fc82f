# bench variants used to locate the executor's cost (see DESIGN.md "Measurements")
set -e
mkdir -p gpurun_out
B="timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
$B > gpurun_out/v_default.log 2>&1
$B --conflict-block 0 > gpurun_out/v_seedmajor.log 2>&1
$B --window 0 --cycle-pct 0 > gpurun_out/v_nopend.log 2>&1
$B --window 4 > gpurun_out/v_w4.log 2>&1
$B --conflicts 0 > gpurun_out/v_c0.log 2>&1
$B --conflicts 100 > gpurun_out/v_c100.log 2>&1
$B --conflicts 100 --window 4 > gpurun_out/v_c100_w4.log 2>&1
