set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
i=0
for kn in "iso_dbg=4" "iso_dbg=36" "iso_dbg=68" "iso_dbg=100" "iso_work_grid=256" "iso_work_grid=256 iso_dbg=4" "iso_work_grid=64 iso_dbg=4"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/fix_$i" -o run -- python3 "$R/tools/iso_fixed_probe.py" 22 $kn > "$R/gpurun_out/fix_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/fix_$i.log"; exit 1; }
  python3 - "$R/gpurun_out/fix_$i/run_kernel_trace.csv" "$kn" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
iso = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_iso_work" in r["Kernel_Name"])
print(f"{sys.argv[2]:32s} s22 k_iso_work n={len(iso)} median {iso[len(iso)//2]:.1f} us min {iso[0]:.1f}")
PY
done
