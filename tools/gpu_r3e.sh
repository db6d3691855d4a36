set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/full.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/full.log | head -20; exit 1; }
bash tools/pmc_passes.sh r03_c2_s22 "k_spmv|k_hot_gather" python3 $GRAFT_REPO_ROOT/tools/spmv_probe.py 22 16 || exit 1
bash tools/pmc_passes.sh r03_msbfs_s22 "k_cw_step|k_cw_hot_gather" python3 $GRAFT_REPO_ROOT/tools/msbfs_probe.py --reps 2 || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --dist-backend gloo --device 0 --scale 18 --steps 4 --warmup 1 --no-cpu-baseline --no-spgemm --no-secondary \
  --msbfs-sharded > gpurun_out/sharded.log 2>&1 || { tail -40 gpurun_out/sharded.log; exit 1; }
grep '^{' gpurun_out/sharded.log | tail -1
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
