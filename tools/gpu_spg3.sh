set -o pipefail
timeout -k 10 200 python3 tools/spgemm_time.py 19 2 "" "spgemm_det=2" "window_order=1" || exit 1
timeout -k 10 200 python3 tools/spgemm_time.py 20 1 "" || exit 1
