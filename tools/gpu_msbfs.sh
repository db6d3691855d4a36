#!/bin/bash
# multi-source BFS: per-level probe, kernel stats, bench line (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/msbfs_probe.py "$@" > gpurun_out/msbfs_probe.log 2>&1 || { tail -30 gpurun_out/msbfs_probe.log; exit 1; }
cat gpurun_out/msbfs_probe.log
bash tools/prof_cmd.sh msbfs_prof python3 tools/msbfs_probe.py "$@" || exit 1
