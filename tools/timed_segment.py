"""Print the kernels of the last BFS of bench.py's timed loop (before the roofline pass's
first GPU spin) from a rocprofv3 kernel-trace csv, with the idle gap before each."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
spins = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
end = spins[0] if spins else len(rows)
seg = rows[max(0, end - n):end]
t0 = int(seg[0]["Start_Timestamp"])
prev = None
busy = 0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    busy += e - s
    print(f"{(s - t0) / 1000:8.1f} gap{gap:6.1f} dur{(e - s) / 1000:7.1f}  {r['Kernel_Name'][:50]}")
    prev = e
print(f"span {(prev - t0) / 1000:.1f} us, kernels busy {busy / 1000:.1f} us")
