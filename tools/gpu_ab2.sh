set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py tests/test_colbits.py -m gpu -q -k "bfs" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tab.log 2>&1; echo tests rc=$?; tail -2 gpurun_out/tab.log
timeout -k 10 400 python3 tools/ab_bfs.py 22 6 "" "pull_steps=1" "pull_steps=-1" "pull_cap=8" "pull_cap=32" "pull_first=1" || exit 1
echo "== HIP_FORCE_DEV_KERNARG=1"
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python3 tools/ab_bfs.py 22 4 "" "pull_steps=1" || exit 1
echo "== HIP_FORCE_DEV_KERNARG=0"
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python3 tools/ab_bfs.py 22 4 "" "pull_steps=1"
