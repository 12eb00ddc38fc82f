# bench variants used to locate the executor's cost (see DESIGN.md "Measurements")
# usage: bash tools/variants.sh [extra bench args, e.g. --tier 0]
mkdir -p gpurun_out && rm -f gpurun_out/v_*.log
B="timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $*"
run() { name=$1; shift; $B "$@" > gpurun_out/v_$name.log 2>&1 || { rc=$?; echo "variant $name rc=$rc"; tail -3 gpurun_out/v_$name.log; exit $rc; }; }
run default
run seedmajor --conflict-block 0
run nopend --window 0 --cycle-pct 0
run w4 --window 4
run c0 --conflicts 0
run c100 --conflicts 100
run c100_w4 --conflicts 100 --window 4
bash tools/show_variants.sh
