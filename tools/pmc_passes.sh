#!/bin/bash
# Per-workload profile for profiles/: one rocprofv3 kernel-trace --stats run, then one
# rocprofv3 --pmc run per counter set (FETCH_SIZE and WRITE_SIZE in separate passes, as
# MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes), restricted to kernels matching a
# regex; then tools/pmc_table.py writes the per-kernel table (gpurun_out/<name>_table.json).
# usage (GPU box, repo root): bash tools/pmc_passes.sh NAME REGEX python3 $GRAFT_REPO_ROOT/tools/x.py args...
set -o pipefail
name=$1; regex=$2; shift 2
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${name}_trace" -o run -- "$@" \
  > "$R/gpurun_out/${name}_trace.log" 2>&1 || { tail -20 "$R/gpurun_out/${name}_trace.log"; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU" ${PMC_EXTRA:+"$PMC_EXTRA"}; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-include-regex "$regex" --pmc $set --output-format csv \
    -d "$R/gpurun_out/${name}_pmc$i" -o run -- "$@" > "$R/gpurun_out/${name}_pmc$i.log" 2>&1 \
    || { tail -5 "$R/gpurun_out/${name}_pmc$i.log"; exit 1; }
done
cd "$R" && python3 tools/pmc_table.py "$name" "$regex"
