#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over the masked-dot probe; kernel filter k_dot
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_dot_task|k_dot_small" --pmc $set --output-format csv -d "$R/gpurun_out/pmc$i" -o run -- python3 "$R/tools/spgemm_probe.py" 20 1 > "$R/gpurun_out/pmc$i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmc$i.log"; exit 1; }
done
echo pmc-done
