# One parameterised GPU session (replaces the per-session tools/exp/r03*.sh drivers).
# Usage (on the box, via gpurun):  bash tools/gpu_session.sh STEP [STEP ...]
# Steps (each under its own time limit; the session stops at the first step
# that crashes, times out or faults -- exit status > 2):
#   test            pytest -m gpu (whole GPU suite)
#   smoke           __graft_entry__.smoke()
#   bench[:ARGS]    python bench.py ARGS  (ARGS: comma-separated, e.g. bench:--config,c2,--steps,20)
#   trace[:ARGS]    rocprofv3 --kernel-trace --hip-runtime-trace of bench.py ARGS (+ timeline.py)
#   ktrace[:ARGS]   rocprofv3 --kernel-trace of bench.py ARGS (+ timeline.py), no runtime trace
#   ctrace[:ARGS]   rocprofv3 --kernel-trace --memory-copy-trace of bench.py ARGS
#   stats[:ARGS]    rocprofv3 --kernel-trace --stats of bench.py ARGS
#   ab:ENV1%ENV2%.. bench lines under each environment (ENVk = A=1+B=2), twice, interleaved; BENCH_ARGS env for the bench flags
#   abl:LIB1%LIB2.. bench lines with each library build (--lib; "default" = the shipped one), twice, interleaved
#   py:SCRIPT,ARGS  python SCRIPT ARGS
# Outputs: gpurun_out/$TAG/<step index>_<name>.{log,json}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-s$(date +%H%M%S)}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  local log="$OUT/$(printf %02d $i)_$name.log"
  echo "== $name: $*" | tee -a "$OUT/session.txt"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.txt"
  tail -3 "$log" | cut -c1-600 | tee -a "$OUT/session.txt"
  if [ $rc -gt 2 ]; then echo "stopping after $name (rc=$rc)" | tee -a "$OUT/session.txt"; exit $rc; fi
  return 0
}
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  IFS=',' read -r -a A <<< "$arg"
  case $kind in
    test)  run test 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "${A[@]}" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py "${A[@]}" ;;
    trace) d="$OUT/trace$i"
           run trace 600 rocprofv3 --kernel-trace --hip-runtime-trace -d "$d" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra "${A[@]}"
           kt=$(find "$d" -name '*kernel_trace.csv' | head -1)
           [ -n "$kt" ] && python3 tools/timeline.py "$kt" 4 > "$OUT/$(printf %02d $i)_timeline.txt" 2>&1 ;;
    ktrace) d="$OUT/ktrace$i"   # kernel trace only (no runtime trace: the host runs at full speed)
           run ktrace 600 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra "${A[@]}"
           kt=$(find "$d" -name '*kernel_trace.csv' | head -1)
           [ -n "$kt" ] && python3 tools/timeline.py "$kt" 4 > "$OUT/$(printf %02d $i)_timeline.txt" 2>&1 ;;
    ctrace) d="$OUT/ctrace$i"   # kernel + memory-copy trace (no runtime trace, no counters)
           run ctrace 600 rocprofv3 --kernel-trace --memory-copy-trace -d "$d" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra "${A[@]}" ;;
    stats) d="$OUT/stats$i"
           run stats 600 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra "${A[@]}" ;;
    ab)    IFS='%' read -r -a ENVS <<< "$arg"
           rep=0
           for e in "${ENVS[@]}" "${ENVS[@]}"; do
             rep=$((rep + 1))
             run "ab$(printf %02d $rep)_${e//[^A-Za-z0-9_=]/_}" 300 env ${e//+/ } python bench.py --no-cpu-baseline --no-extra --steps ${STEPS:-100} --warmup 10 $BENCH_ARGS
           done ;;
    abl)   IFS='%' read -r -a LIBS <<< "$arg"   # library builds (default = the shipped one), twice, interleaved
           rep=0
           for l in "${LIBS[@]}" "${LIBS[@]}"; do
             rep=$((rep + 1))
             la=""; [ "$l" != "default" ] && la="--lib $l"
             run "abl$(printf %02d $rep)_$(basename "$l" .so)" 300 python bench.py --no-cpu-baseline --no-extra --steps ${STEPS:-100} --warmup ${WARM:-50} $la $BENCH_ARGS
           done ;;
    py)    run "py_$(basename "${A[0]}" .py)" 600 python "${A[@]}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done" | tee -a "$OUT/session.txt"
