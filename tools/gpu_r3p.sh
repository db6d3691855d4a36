set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_end" -o bench -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_end.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_end.log"; exit 1; }
cd "$R" && python3 tools/kstats.py gpurun_out/prof_end/bench_kernel_stats.csv | head -12
grep '^{' gpurun_out/prof_end.log | tail -1 | cut -c1-300
