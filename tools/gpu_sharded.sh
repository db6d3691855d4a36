#!/bin/bash
# batched-frontier tests, then a 2-rank gloo rehearsal of the sharded multi-source BFS on
# one GPU (both ranks on device 0; the exchange stages through host memory)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_colbits.py -x -q --timeout 120 --timeout-method thread > gpurun_out/colbits_tests.log 2>&1 || { tail -40 gpurun_out/colbits_tests.log; exit 1; }
tail -1 gpurun_out/colbits_tests.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --dist-backend gloo --device 0 --scale ${1:-18} --steps 4 --warmup 1 --no-cpu-baseline --no-spgemm \
  --msbfs-sharded > gpurun_out/sharded.log 2>&1 || { tail -40 gpurun_out/sharded.log; exit 1; }
grep '^{' gpurun_out/sharded.log | tail -1
