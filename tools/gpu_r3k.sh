set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_bfs.py 22 10 "" "iso_occ=6" "iso_occ=8" || exit 1
