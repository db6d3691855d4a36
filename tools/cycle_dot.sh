set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "two_sided or masked_spgemm or random_mxm or deferred" > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 120 python tools/spgemm_probe.py 20 3 > gpurun_out/probe20.log 2>&1 || { tail -20 gpurun_out/probe20.log; exit 1; }
cat gpurun_out/probe20.log
timeout -k 10 120 python tools/spgemm_probe.py 22 2 >> gpurun_out/probe20.log 2>&1 || { tail -20 gpurun_out/probe20.log; exit 1; }
tail -1 gpurun_out/probe20.log
