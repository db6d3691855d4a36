"""Sum rocprofv3 PMC counters per kernel over the passes <prefix>1..N (counter_collection.csv)."""
import collections
import csv
import glob
import sys

prefix = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for d in sorted(glob.glob(prefix + "*/")):
    for f in glob.glob(d + "*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:22s} {v:.4g}")
