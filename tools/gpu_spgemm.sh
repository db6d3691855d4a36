set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_spgemm_det.py tests/test_gpu_parity.py -m gpu -x -q -s -k "spgemm or det" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tsp.log 2>&1; rc=$?; echo tests rc=$rc; grep -E "differ|passed|failed|Error" gpurun_out/tsp.log | tail -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 tools/spgemm_time.py 19 3 "" "spgemm_det=2" "window_order=1"
