# round-6 secondary profiles of the final tree (tools/pmc_passes.sh per workload; tools/pmc_percall.py
# turns each into profiles/r06_<workload>_pmc.json on the CPU side)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
bash tools/pmc_passes.sh c2s22 'k_spmv|k_hot' python3 "$R/tools/spmv_probe.py" 22 16 || exit 1
bash tools/pmc_passes.sh c2s22e60 'k_spmv|k_hot' python3 "$R/tools/spmv_probe.py" 22 60 || exit 1
bash tools/pmc_passes.sh c5s19 'k_|Segmented|Radix|radix' python3 "$R/tools/spgemm_time.py" 19 1 || exit 1
bash tools/pmc_passes.sh c5s20 'k_|Segmented|Radix|radix' python3 "$R/tools/spgemm_time.py" 20 1 || exit 1
bash tools/pmc_passes.sh msbfs 'k_cw_step|k_cw_hot_gather' python3 "$R/tools/msbfs_probe.py" --reps 2 || exit 1
bash tools/pmc_passes.sh c4s22 k_d python3 "$R/tools/spgemm_probe.py" 22 1 || exit 1
bash tools/pmc_passes.sh c4s20 k_d python3 "$R/tools/spgemm_probe.py" 20 1 || exit 1
bash tools/pmc_kernel.sh c4task k_dot_task python3 "$R/tools/spgemm_probe.py" 22 1 || exit 1
echo callB-ok
