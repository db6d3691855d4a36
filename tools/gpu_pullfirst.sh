set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py -m gpu -q -k "bfs" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tpf.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/tpf.log
for pf in 0 1; do
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-secondary --no-msbfs --no-spgemm --no-cpu-baseline --knob pull_first=$pf > gpurun_out/bpf$pf.json 2>gpurun_out/bpf$pf.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bpf$pf.json').read().splitlines()[-1]);print('pull_first knob',$pf,d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
done
timeout -k 10 200 python3 tools/level_probe.py 22 7 > gpurun_out/lvl0.txt 2>&1; tail -25 gpurun_out/lvl0.txt
