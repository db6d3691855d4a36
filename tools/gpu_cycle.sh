#!/bin/bash
# One GPU cycle: parity tests, bench, kernel-trace profile.  Run via gpurun from the repo root.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 8 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
echo profiled
