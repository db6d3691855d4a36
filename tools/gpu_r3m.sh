set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_gpu.py -m gpu -x -q -k "bfs or sharded or deferred or iso or random_spmv" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t.log | head -20; exit 1; }
timeout -k 10 300 python3 tools/ab_bfs.py 22 10 "" || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/fixB" -o run -- python3 "$GRAFT_REPO_ROOT/tools/iso_fixed_probe.py" 22 > "$GRAFT_REPO_ROOT/gpurun_out/fixB.log" 2>&1 || exit 1
python3 - "$GRAFT_REPO_ROOT/gpurun_out/fixB/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
iso = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_iso_work" in r["Kernel_Name"])
print(f"one-vertex level s22 k_iso_work n={len(iso)} median {iso[len(iso)//2]:.1f} us min {iso[0]:.1f}")
PY
