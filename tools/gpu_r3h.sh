set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "spgemm or mxm or dot" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
timeout -k 10 200 python3 tools/spgemm_probe.py 20 3 || exit 1
timeout -k 10 300 python3 tools/spgemm_probe.py 22 2 || exit 1
