"""Per-kernel table of one tools/pmc_passes.sh run: launches and average duration from the
kernel-trace stats, per-dispatch means of every PMC counter, and HBM bytes per launch =
2 x FETCH_SIZE (gfx950: FETCH_SIZE counts half the bytes of wide streaming reads,
MI355X_MICROARCH.md HBM/rocprofv3) + WRITE_SIZE, both KiB.  Writes
gpurun_out/<name>_table.json and prints it.
usage: python3 tools/pmc_table.py NAME [REGEX]"""
import collections
import csv
import glob
import json
import os
import re
import sys

name = sys.argv[1]
regex = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = os.path.join(root, "gpurun_out")


def short(k):
    k = k.replace("(anonymous namespace)::", "").replace("void ", "")
    # keep template arguments, drop the parameter list
    depth, cut = 0, len(k)
    for i, ch in enumerate(k):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return k[:cut].strip()


stats = {}
for f in glob.glob(os.path.join(out_dir, f"{name}_trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        k = short(r["Name"])
        if regex and not regex.search(k):
            continue
        s = stats.setdefault(k, {"launches": 0, "total_ns": 0.0})
        s["launches"] += int(r["Calls"])
        s["total_ns"] += float(r["TotalDurationNs"])
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(out_dir, f"{name}_pmc*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
table = {}
for (k, c), v in vals.items():
    t = table.setdefault(k, {})
    t[c] = sum(v) / len(v)
    t[c + "_dispatches"] = len(v)
for k, t in table.items():
    if k in stats:
        t["launches"] = stats[k]["launches"]
        t["avg_us"] = stats[k]["total_ns"] / stats[k]["launches"] / 1e3
    if "FETCH_SIZE" in t:
        t["hbm_bytes_per_launch"] = 2 * t["FETCH_SIZE"] * 1024 + t.get("WRITE_SIZE", 0.0) * 1024
    if "TCC_HIT_sum" in t and t["TCC_HIT_sum"] + t.get("TCC_MISS_sum", 0) > 0:
        t["l2_hit"] = t["TCC_HIT_sum"] / (t["TCC_HIT_sum"] + t["TCC_MISS_sum"])
    if t.get("SQ_WAVE_CYCLES"):
        t["wait_frac"] = t.get("SQ_WAIT_ANY", 0) / t["SQ_WAVE_CYCLES"]
res = {"name": name, "regex": regex.pattern if regex else None,
       "method": "rocprofv3 --kernel-trace --stats, then one --pmc pass per counter set; hbm_bytes_per_launch = "
                 "2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes, gfx950 FETCH correction)",
       "kernels": table, "trace_stats": stats}
json.dump(res, open(os.path.join(out_dir, f"{name}_table.json"), "w"), indent=1)
for k, t in sorted(table.items(), key=lambda kv: -kv[1].get("avg_us", 0) * kv[1].get("launches", 0)):
    print(f"{k[:60]:60s} n={t.get('launches')} avg_us={t.get('avg_us', 0):.1f} "
          f"hbm/launch={t.get('hbm_bytes_per_launch', 0) / 1e6:.1f}MB l2hit={t.get('l2_hit', 0):.2f} "
          f"wait={t.get('wait_frac', 0):.2f}")
