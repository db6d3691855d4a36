set -o pipefail
timeout -k 10 200 python3 tools/iso_probe.py 22 "spmv_direction=2" "spmv_direction=2,iso_work_grid=512" "spmv_direction=2,iso_work_grid=256" "spmv_direction=2,iso_work_grid=128" "spmv_direction=2,iso_work_grid=64" "spmv_direction=2,iso_dbg=9" "spmv_direction=2,iso_dbg=9,iso_work_grid=128" "spmv_direction=2,iso_dbg=5" "spmv_direction=2,iso_dbg=5,iso_work_grid=128" "spmv_direction=2,iso_dbg=1" || exit 1
timeout -k 10 300 python3 tools/ab_bfs.py 22 4 "" "iso_work_grid=512" "iso_work_grid=2048" || exit 1
