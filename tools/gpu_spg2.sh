set -o pipefail
for sc in 14 16 17; do
  timeout -k 10 100 python3 tools/spgemm_time.py $sc 2 "" "spgemm_det=2" || exit 1
done
