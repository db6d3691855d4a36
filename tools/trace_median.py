"""Median duration (us) of the kernels matching a regex in a rocprofv3 kernel_trace csv."""
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2])
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if pat.search(r["Kernel_Name"])]
print(f"{sys.argv[2]}: n={len(d)} median={statistics.median(d):.2f}us min={min(d):.2f}us" if d else "none")
