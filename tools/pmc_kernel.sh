#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) of one command, restricted to kernels
# matching a regex; then a per-kernel summary.
# usage (GPU box, repo root): bash tools/pmc_kernel.sh NAME REGEX python3 $GRAFT_REPO_ROOT/tools/x.py args...
set -o pipefail
name=$1; regex=$2; shift 2
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$regex" --pmc $set --output-format csv -d "$R/gpurun_out/${name}_pmc$i" -o run -- "$@" > "$R/gpurun_out/${name}_pmc$i.log" 2>&1 || { tail -5 "$R/gpurun_out/${name}_pmc$i.log"; exit 1; }
done
cd "$R" && python3 tools/pmc_summary.py gpurun_out/${name}_pmc
