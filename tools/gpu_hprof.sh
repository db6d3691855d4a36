set -o pipefail
GRAPHBLAS_AMD_HPROF=1 timeout -k 10 300 python3 tools/ab_bfs.py 22 6 "" 2>&1 | tail -20
