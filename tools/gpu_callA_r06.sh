set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/collect_profiles.sh || exit 1
bash tools/pmc_passes.sh c4s22 k_d python3 "$GRAFT_REPO_ROOT/tools/spgemm_probe.py" 22 1 || exit 1
bash tools/pmc_passes.sh c4s20 k_d python3 "$GRAFT_REPO_ROOT/tools/spgemm_probe.py" 20 1 || exit 1
bash tools/pmc_kernel.sh c4task k_dot_task python3 "$GRAFT_REPO_ROOT/tools/spgemm_probe.py" 22 1 || exit 1
echo callA-ok
