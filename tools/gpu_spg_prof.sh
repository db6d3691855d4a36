# kernel stats of the config-5 SpGEMM (tools/spgemm_time.py) under knob settings; GPU box
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
sc=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/spg_prof_s$sc" -o run -- python3 "$R/tools/spgemm_time.py" $sc 1 "$@" > "$R/gpurun_out/spg_prof_s$sc.log" 2>&1 || { tail -20 "$R/gpurun_out/spg_prof_s$sc.log"; exit 1; }
cd "$R" && grep "\[" gpurun_out/spg_prof_s$sc.log | tail -4
python3 - "$R/gpurun_out/spg_prof_s$sc" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:10.1f} us  {r['Name'][:120]}")
PY
