"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (name, calls, avg, total)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:top]:
    print(f"{r['Name'][:100]:100s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.1f}us "
          f"{float(r['TotalDurationNs']) / 1e6:9.2f}ms")
