set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_colbits.py -x -v --timeout 120 --timeout-method thread > gpurun_out/colbits_tests.log 2>&1 || { tail -40 gpurun_out/colbits_tests.log; exit 1; }
tail -1 gpurun_out/colbits_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-secondary --no-spgemm > gpurun_out/bench_ms.log 2>&1 || { tail -30 gpurun_out/bench_ms.log; exit 1; }
tail -1 gpurun_out/bench_ms.log
