#!/bin/bash
# Round profile collection on the GPU box (run from the repo root via gpurun):
#   1. default bench (with cpu_baseline) -> gpurun_out/bench_full.json
#   2. rocprofv3 --kernel-trace --stats of the bench -> gpurun_out/prof_stats/
#   3. PMC passes (FETCH_SIZE, then WRITE_SIZE; separate passes) on the BFS kernels -> gpurun_out/pmc_*/
set -o pipefail
R=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_stats" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_stats.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_stats.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_iso_work|k_assign_mask_words" --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_iso_work|k_assign_mask_words" --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.log"; exit 1; }
echo collected
