#!/bin/bash
# One GPU-box call as a chain of named steps (replaces the per-round one-off gpu_*.sh scripts).
# Every step has its own time limit; the chain stops at the first failing step.
# usage (via gpurun, from the repo root):
#   bash tools/gpu_steps.sh STEP [STEP ...]
# steps:
#   tests                 the whole -m gpu suite               -> gpurun_out/tests.log
#   tests:EXPR            -m gpu tests selected by -k EXPR     -> gpurun_out/tests_<n>.log
#   file:PATH             -m gpu tests of one file             -> gpurun_out/tests_<n>.log
#   smoke                 __graft_entry__.smoke()
#   bench                 bench.py with its defaults           -> gpurun_out/bench.log (+ bench.json)
#   bench:ARGS            bench.py ARGS (comma-separated)      -> gpurun_out/bench_<n>.log
#   stats:NAME            rocprofv3 --kernel-trace --stats of the default bench (no CPU baseline)
#                         -> gpurun_out/NAME/ + top kernels (tools/kstats.py)
#   prof:NAME:CMD         the same for CMD (comma-separated argv: a script under the repo root + args)
#   roctx:NAME:CMD        kernel trace + roctx ranges per library call (tools/prof_roctx.sh)
#   pmc:NAME:REGEX:CMD    tools/pmc_passes.sh NAME REGEX CMD (trace + FETCH / WRITE / TCC / SQ passes)
#   pmck:NAME:REGEX:CMD   tools/pmc_kernel.sh NAME REGEX CMD (instruction mix, LDS, waits, L2, FETCH)
#   py:CMD                python3 CMD (comma-separated argv), 300 s limit
#   pyx:CMD               the same with ~ separating the arguments (arguments that hold commas)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
n=0
PYT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  echo "== step $n: $step"
  case $kind in
  tests)
    if [ -z "$rest" ]; then
      timeout -k 10 900 $PYT tests > gpurun_out/tests.log 2>&1; rc=$?; log=gpurun_out/tests.log
    else
      timeout -k 10 600 $PYT tests -k "$rest" > gpurun_out/tests_$n.log 2>&1; rc=$?; log=gpurun_out/tests_$n.log
    fi
    tail -3 $log
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $log | head -20; exit 1; } ;;
  file)
    timeout -k 10 600 $PYT -v "$rest" > gpurun_out/tests_$n.log 2>&1; rc=$?
    tail -4 gpurun_out/tests_$n.log
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/tests_$n.log | head -20; exit 1; } ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
  bench)
    if [ -z "$rest" ]; then
      timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
      grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench.json
      cut -c1-400 gpurun_out/bench.json
    else
      timeout -k 10 600 python3 bench.py ${rest//,/ } > gpurun_out/bench_$n.log 2>&1 || { tail -20 gpurun_out/bench_$n.log; exit 1; }
      grep '^{' gpurun_out/bench_$n.log | tail -1 | cut -c1-400
    fi ;;
  stats)
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$rest" -o bench \
      -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/$rest.log" 2>&1) || { tail -20 "gpurun_out/$rest.log"; exit 1; }
    python3 tools/kstats.py "gpurun_out/$rest/bench_kernel_stats.csv" | head -16
    grep '^{' "gpurun_out/$rest.log" | tail -1 > "gpurun_out/$rest.json" ;;
  prof)
    name=${rest%%:*}; cmd=${rest#*:}
    argv=(${cmd//,/ })
    bash tools/prof_cmd.sh "$name" python3 "$R/${argv[0]}" "${argv[@]:1}" || exit 1 ;;
  roctx)
    name=${rest%%:*}; cmd=${rest#*:}
    argv=(${cmd//,/ })
    bash tools/prof_roctx.sh "$name" python3 "$R/${argv[0]}" "${argv[@]:1}" || exit 1 ;;
  pmc)
    name=${rest%%:*}; r2=${rest#*:}; regex=${r2%%:*}; cmd=${r2#*:}
    argv=(${cmd//,/ })
    bash tools/pmc_passes.sh "$name" "$regex" python3 "$R/${argv[0]}" "${argv[@]:1}" || exit 1 ;;
  pmck)
    name=${rest%%:*}; r2=${rest#*:}; regex=${r2%%:*}; cmd=${r2#*:}
    argv=(${cmd//,/ })
    bash tools/pmc_kernel.sh "$name" "$regex" python3 "$R/${argv[0]}" "${argv[@]:1}" || exit 1 ;;
  py)
    timeout -k 10 300 python3 ${rest//,/ } || exit 1 ;;
  pyx)
    IFS='~' read -r -a argv <<< "$rest"
    timeout -k 10 300 python3 "${argv[@]}" || exit 1 ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps ok"
