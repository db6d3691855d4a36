set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/spmv_ab.py 22 16 6 "" "spmv_nt=1" "spmv_words=2" "spmv_words=2,spmv_nt=1" || exit 1
timeout -k 10 300 python3 tools/spmv_ab.py 22 60 4 "" "spmv_nt=1" || exit 1
timeout -k 10 400 python3 tools/spgemm_time.py 20 1 || exit 1
