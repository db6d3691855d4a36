set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_spg_prof.sh 19 || exit 1
timeout -k 10 400 python3 tools/spgemm_time.py 19 2 "" "window_in_c_groups=3" "window_in_c_groups=24" "window_bits=1" || exit 1
for r in 7 3 11; do timeout -k 10 120 python3 tools/level_probe.py 22 $r > gpurun_out/lvl$r.txt 2>&1 || { tail -5 gpurun_out/lvl$r.txt; exit 1; }; grep -A10 "out-degree" gpurun_out/lvl$r.txt; done
