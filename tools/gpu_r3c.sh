set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_spg_prof.sh 19 || exit 1
timeout -k 10 300 python -u tools/msbfs_probe.py > gpurun_out/msbfs_probe.log 2>&1 || { tail -30 gpurun_out/msbfs_probe.log; exit 1; }
cat gpurun_out/msbfs_probe.log
