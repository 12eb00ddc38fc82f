# One GPU-box call made of steps, run in order; the call stops at the first
# step that fails (a fault, abort or time limit ends it at once, as the pool's
# rules ask).  Every step has its own time limit and writes its log under OUT.
#
# usage (from the repo root of the box, e.g. through gpurun):
#   OUT=gpurun_out/r6b bash tools/gpu_call.sh "STEP ARGS..." ["STEP ARGS..." ...]
# steps:
#   tests [pytest args]        GPU tests (default: the whole -m gpu suite)
#   smoke                      __graft_entry__.smoke()
#   bench NAME [bench args]    python bench.py ARGS -> NAME.log (prints the line's headline numbers)
#   ab NAME LIB [bench args]   the same with FX_LIB=LIB (a library variant: make fvariant / variant)
#   trace NAME [bench args]    rocprofv3 --kernel-trace --stats of the bench -> NAME/
#   pmc MODE PATTERN [args]    the counter passes of one bench mode's kernel (tools/mode_pmc.sh;
#                              outputs under gpurun_out/pmc_MODE/)
#   py NAME SCRIPT [args]      python3 -u SCRIPT ARGS -> NAME.log (diagnostics under tools/)
# env: OUT (default gpurun_out/call), T_TESTS / T_BENCH / T_PY (seconds)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/call}
mkdir -p "$OUT"
T_TESTS=${T_TESTS:-900}
T_BENCH=${T_BENCH:-400}
T_PY=${T_PY:-600}

line() {  # the headline fields of a bench JSON line
  python3 -c "import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print('%-14s %s %.4g %s  %.2f ms/step  frac %s  traffic %s' % (sys.argv[2], d['metric'][:28], d['value'], d['unit'],
      d['ms_per_step'], r.get('frac'), r.get('traffic_over_alg')))" "$1" "$2"
}

step() {
  local kind=$1; shift
  case $kind in
    tests)
      local args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
      timeout -k 10 "$T_TESTS" python3 -u -m pytest -x -q --timeout 300 --timeout-method thread "${args[@]}" \
        > "$OUT/tests.log" 2>&1
      local rc=$?; tail -3 "$OUT/tests.log"; return $rc ;;
    smoke)
      timeout -k 10 300 python3 -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
      local rc=$?; tail -2 "$OUT/smoke.log"; return $rc ;;
    bench)
      local nm=$1; shift
      timeout -k 10 "$T_BENCH" python3 bench.py "$@" > "$OUT/$nm.log" 2>&1
      local rc=$?; [ $rc -eq 0 ] && line "$OUT/$nm.log" "$nm" || tail -5 "$OUT/$nm.log"; return $rc ;;
    ab)
      local nm=$1 lib=$2; shift 2
      FX_LIB=$lib timeout -k 10 "$T_BENCH" python3 bench.py "$@" > "$OUT/$nm.log" 2>&1
      local rc=$?; [ $rc -eq 0 ] && line "$OUT/$nm.log" "$nm" || tail -5 "$OUT/$nm.log"; return $rc ;;
    trace)
      local nm=$1; shift
      timeout -k 10 "$T_BENCH" rocprofv3 --kernel-trace --stats -d "$OUT/$nm" -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline "$@" > "$OUT/$nm.log" 2>&1
      local rc=$?; find "$OUT/$nm" -name "*kernel_stats.csv" | head -1 | xargs -r head -4; return $rc ;;
    pmc)
      bash tools/mode_pmc.sh "$@"; return $? ;;
    py)
      local nm=$1 script=$2; shift 2
      timeout -k 10 "$T_PY" python3 -u "$script" "$@" > "$OUT/$nm.log" 2>&1
      local rc=$?; tail -15 "$OUT/$nm.log"; return $rc ;;
    *) echo "unknown step: $kind"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  # shellcheck disable=SC2086
  step $s
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "step '$s' failed (rc $rc): the call stops here"
    exit $rc
  fi
done
