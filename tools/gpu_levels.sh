# per-level BFS timings (tools/level_probe.py) under knob settings, the BFS parity tests and a
# short headline bench with the pull heads on / off; GPU box, repo root
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py tests/test_colbits.py -m gpu -q -k "bfs" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tpf.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/tpf.log
for kv in "" "frontier_summary=1" "pull_first=1"; do
  echo "== knobs: $kv"
  timeout -k 10 120 python3 tools/level_probe.py 22 7 $kv > gpurun_out/lvl.txt 2>&1 || { tail -5 gpurun_out/lvl.txt; exit 1; }
  grep -A9 " lvl" gpurun_out/lvl.txt
done
for pf in 0 1; do  # knob frontier_summary
  timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-secondary --no-msbfs --no-spgemm --no-cpu-baseline --knob frontier_summary=$pf > gpurun_out/bpf$pf.json 2>gpurun_out/bpf$pf.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bpf$pf.json').read().splitlines()[-1]);print("frontier_summary knob",$pf,d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d['roofline']['frac'])"
done
