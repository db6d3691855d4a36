# round-6 final tree: config 4 profiles (its kernels changed last), then the whole -m gpu suite,
# the default bench and smoke() -- tools/pmc_percall.py writes profiles/r06_config4_*_pmc.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
bash tools/pmc_passes.sh c4s22 k_d python3 "$R/tools/spgemm_probe.py" 22 1 || exit 1
bash tools/pmc_passes.sh c4s20 k_d python3 "$R/tools/spgemm_probe.py" 20 1 || exit 1
bash tools/pmc_kernel.sh c4task k_dot_task python3 "$R/tools/spgemm_probe.py" 22 1 || exit 1
bash tools/gpu_callC_r06.sh || exit 1
echo final-ok
