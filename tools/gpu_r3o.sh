set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/spmv_ab.py 22 16 6 "" "spmv_nt=1" "spmv_words=2" "spmv_nt=1,spmv_words=2" > gpurun_out/spmv_ab16.txt 2>&1 || { tail -5 gpurun_out/spmv_ab16.txt; exit 1; }
cat gpurun_out/spmv_ab16.txt | tail -8
timeout -k 10 300 python3 tools/spmv_ab.py 22 60 4 "" "spmv_nt=1" "spmv_words=2" > gpurun_out/spmv_ab60.txt 2>&1 || { tail -5 gpurun_out/spmv_ab60.txt; exit 1; }
cat gpurun_out/spmv_ab60.txt | tail -8
