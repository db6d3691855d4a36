set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py -m gpu -x -q -k "bfs or sharded or deferred" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
for a in 8 4 16 32; do timeout -k 10 200 python -u tools/msbfs_probe.py --knob colbits_alpha=$a --reps 4 > gpurun_out/ms$a.log 2>&1 || { tail -5 gpurun_out/ms$a.log; exit 1; }; echo "colbits_alpha=$a $(grep 'batch wall' gpurun_out/ms$a.log)"; done
timeout -k 10 300 python3 tools/ab_bfs.py 22 8 "" "push_alpha=14" "push_heavy=256" || exit 1
