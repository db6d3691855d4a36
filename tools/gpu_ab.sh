# A/B of BFS knob settings in one process (tools/ab_bfs.py) after the BFS parity tests; GPU box
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py tests/test_colbits.py -m gpu -q -k "bfs" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tab.log 2>&1; echo tests rc=$?; tail -2 gpurun_out/tab.log
timeout -k 10 400 python3 tools/ab_bfs.py 22 ${ROUNDS:-8} "$@"
