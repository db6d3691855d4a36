set -o pipefail
bash tools/gpu_spg4.sh || exit 1
echo "== BFS kernel trace"
bash tools/gpu_trace_bfs.sh > gpurun_out/trace_bfs.txt 2>&1; echo trace rc=$?; tail -62 gpurun_out/trace_bfs.txt
