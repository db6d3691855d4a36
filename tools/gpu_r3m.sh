set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py -m gpu -x -q -k "bfs or sharded or deferred or iso or fused" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
timeout -k 10 300 python3 tools/ab_bfs.py 22 10 "" || exit 1
bash tools/gpu_trace_bfs.sh > gpurun_out/trace.txt 2>&1 || { tail -5 gpurun_out/trace.txt; exit 1; }
grep -c k_dir_prep gpurun_out/trace.txt; grep -c k_iso_work gpurun_out/trace.txt
