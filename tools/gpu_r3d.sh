set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_colbits.py -m gpu -x -q -k "hot_columns or spmv or msbfs" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
timeout -k 10 200 python3 tools/xhot_probe.py 22 16 65536 262144 524288 1048576 || exit 1
timeout -k 10 200 python3 tools/xhot_probe.py 22 60 262144 524288 1048576 || exit 1
timeout -k 10 200 python -u tools/msbfs_probe.py --knob colbits_hot=1 > gpurun_out/msbfs_probe0.log 2>&1 || { tail -30 gpurun_out/msbfs_probe0.log; exit 1; }
timeout -k 10 200 python -u tools/msbfs_probe.py > gpurun_out/msbfs_probe1.log 2>&1 || { tail -30 gpurun_out/msbfs_probe1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/msbfs_probe0.log; grep -v amdgpu.ids gpurun_out/msbfs_probe1.log
