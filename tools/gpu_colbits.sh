#!/bin/bash
# batched-frontier parity tests, then the per-level probe (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_colbits.py -x -q --timeout 120 --timeout-method thread > gpurun_out/colbits_tests.log 2>&1 || { tail -40 gpurun_out/colbits_tests.log; exit 1; }
tail -1 gpurun_out/colbits_tests.log
for al in "$@"; do
timeout -k 10 200 python -u tools/msbfs_probe.py --knob colbits_alpha=$al > gpurun_out/msbfs_probe_$al.log 2>&1 || { tail -30 gpurun_out/msbfs_probe_$al.log; exit 1; }
echo "alpha $al"; grep -v amdgpu.ids gpurun_out/msbfs_probe_$al.log
done
