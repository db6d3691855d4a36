#!/bin/bash
# rocprofv3 kernel trace + roctx ranges (GRAPHBLAS_AMD_ROCTX=1: every GrB_*/GxB_* entry point
# pushes a range named after itself) of one command, so each kernel can be attributed to the
# library call that launched it (tools/roctx_attrib.py).  No PMC counters in this run.
# usage (GPU box, repo root): bash tools/prof_roctx.sh NAME python3 $GRAFT_REPO_ROOT/x.py args...
set -o pipefail
name=$1; shift
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
export GRAPHBLAS_AMD_ROCTX=1
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --stats --output-format csv -d "$R/gpurun_out/$name" -o run \
  -- "$@" > "$R/gpurun_out/$name.log" 2>&1 || { tail -30 "$R/gpurun_out/$name.log"; exit 1; }
cd "$R" && ls gpurun_out/$name && python3 tools/roctx_attrib.py gpurun_out/$name | head -40
