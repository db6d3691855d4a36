# kernel trace of the headline BFS loop (tools/ab_bfs.py, 1 round, defaults): per-dispatch start/duration
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_bfs" -o run -- python3 "$R/tools/ab_bfs.py" 22 1 "$@" > "$R/gpurun_out/trace_bfs.log" 2>&1 || { tail -20 "$R/gpurun_out/trace_bfs.log"; exit 1; }
cd "$R" && tail -2 gpurun_out/trace_bfs.log && python3 tools/timeline.py gpurun_out/trace_bfs/run_kernel_trace.csv 60
