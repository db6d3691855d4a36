#!/bin/bash
# Round profile collection on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench (no CPU baseline) -> gpurun_out/prof_stats/
#   2. the BFS-only bench with the level speculation off: kernel stats (prof_stats_nospec) and PMC
#      passes (FETCH_SIZE, then WRITE_SIZE; separate passes) on the headline BFS kernels
#      -> gpurun_out/pmc_*/; tools/summarize_profiles.py turns them into profiles/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_stats" -o bench -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_stats.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_stats.log"; exit 1; }
grep '^{' "$R/gpurun_out/prof_stats.log" | tail -1 > "$R/gpurun_out/prof_bench.json"
# the BFS alone with the level speculation off (knob bfs_spec=1): one k_iso_work launch per
# level, as the bench's event-bracketed roofline pass times them (with speculation on, each BFS
# adds one empty launch for the level after its last)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_stats_nospec" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --no-secondary --no-msbfs --no-spgemm --knob bfs_spec=1 > "$R/gpurun_out/prof_stats_nospec.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_stats_nospec.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | tr 'A-Z' 'a-z' | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --kernel-include-regex "k_iso_work|k_dir_prep" --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$lc" -o bench -- python3 "$R/bench.py" --no-cpu-baseline --no-secondary --no-msbfs --no-spgemm --knob bfs_spec=1 > "$R/gpurun_out/pmc_$lc.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_$lc.log"; exit 1; }
done
echo collected
