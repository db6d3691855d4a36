#!/bin/bash
# rocprofv3 kernel-trace stats of one command; prints the top kernels.
# usage (on the GPU box, from the repo root): bash tools/prof_cmd.sh NAME python3 tools/x.py args...
set -o pipefail
name=$1; shift
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$name" -o run -- "$@" > "$R/gpurun_out/$name.log" 2>&1 || { tail -30 "$R/gpurun_out/$name.log"; exit 1; }
cd "$R" && python3 tools/kstats.py "gpurun_out/$name/run_kernel_stats.csv"
