set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/full.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/full.log | head -20; exit 1; }
bash tools/gpu_trace_bfs.sh
