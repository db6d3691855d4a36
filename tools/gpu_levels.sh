# per-level BFS timings (tools/level_probe.py) under several knob settings; GPU box, repo root
set -o pipefail
for kv in "" "pull_first=1" "iso_dbg=16" "iso_dbg=32" "pull_steps=-1" "iso_dbg=48"; do
  echo "== knobs: $kv"
  timeout -k 10 120 python3 tools/level_probe.py 22 7 $kv > gpurun_out/lvl.txt 2>&1 || { tail -5 gpurun_out/lvl.txt; exit 1; }
  grep -A9 " lvl" gpurun_out/lvl.txt
done
