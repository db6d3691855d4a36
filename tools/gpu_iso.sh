set -o pipefail
timeout -k 10 200 python3 tools/iso_probe.py 22 "" "iso_dbg=1" "iso_dbg=3" "iso_dbg=5" "iso_dbg=9" "spmv_direction=2" "spmv_direction=2,iso_dbg=5" "spmv_direction=1" "spmv_direction=1,iso_dbg=5"
