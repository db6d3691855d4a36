set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_spgemm_det.py -m gpu -x -q -k "hash or spgemm or det" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
timeout -k 10 300 python3 tools/spgemm_time.py 19 3 || exit 1
bash tools/pmc_passes.sh r03_c4_s22 "k_dot|k_dt_" python3 $GRAFT_REPO_ROOT/tools/spgemm_probe.py 22 1 || exit 1
