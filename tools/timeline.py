"""Print the last N kernel dispatches of a rocprofv3 --kernel-trace csv (start offset, duration, name)."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  grid={int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])):6d}  {r['Kernel_Name'][:70]}")
