set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/full.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/full.log | head -5; exit 1; }
timeout -k 10 300 python3 tools/ab_bfs.py 22 6 "" "zero_pool=1" "host_dir=1" "zero_pool=1,host_dir=1" || exit 1
