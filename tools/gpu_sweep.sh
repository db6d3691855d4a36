#!/bin/bash
# sweep one knob of the multi-source BFS probe: bash tools/gpu_sweep.sh KNOB v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
knob=$1; shift
for v in "$@"; do
timeout -k 10 200 python -u tools/msbfs_probe.py --knob $knob=$v > gpurun_out/sweep_$v.log 2>&1 || { tail -30 gpurun_out/sweep_$v.log; exit 1; }
echo "$knob $v"; grep -v amdgpu.ids gpurun_out/sweep_$v.log
done
