"""Turn a round's rocprofv3 outputs (tools/collect_profiles.sh) into the committed
profiles/: kernel stats, per-kernel PMC means and traffic_<round>.json.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and
WRITE_SIZE are collected in separate passes (units: KiB); on gfx950 FETCH_SIZE counts
half the bytes of wide streaming reads, so it is doubled before use."""
import collections
import csv
import json
import os
import shutil
import sys

rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out")
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "prof_stats", "bench_kernel_stats.csv"), os.path.join(dst, f"{rnd}_bench_kernel_stats.csv"))


def means(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: (len(v), sum(v) / len(v)) for k, v in agg.items()}


fetch = means(os.path.join(src, "pmc_fetch", "bench_counter_collection.csv"))
write = means(os.path.join(src, "pmc_write", "bench_counter_collection.csv"))
# per-launch durations from the run the PMC passes repeat (speculation off: one launch per level)
sdir = "prof_stats_nospec" if os.path.isdir(os.path.join(src, "prof_stats_nospec")) else "prof_stats"
if sdir == "prof_stats_nospec":
    shutil.copy(os.path.join(src, sdir, "bench_kernel_stats.csv"), os.path.join(dst, f"{rnd}_bfs_nospec_kernel_stats.csv"))
stats = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(os.path.join(src, sdir, "bench_kernel_stats.csv")))}
lines = ["kernel,launches,avg_us,FETCH_SIZE_KiB_mean,WRITE_SIZE_KiB_mean,hbm_bytes_per_launch_corrected"]
out = {}
for (kname, _), (cnt, fkib) in fetch.items():
    wkib = write.get((kname, "WRITE_SIZE"), (0, 0.0))[1]
    corrected = fkib * 1024 * 2 + wkib * 1024
    avg_us = float(stats[kname]["AverageNs"]) / 1e3 if kname in stats else None
    lines.append(f"{kname},{cnt},{avg_us},{fkib:.1f},{wkib:.1f},{corrected:.0f}")
    out[kname] = {"launches": cnt, "avg_us": avg_us, "fetch_kib": fkib, "write_kib": wkib, "bytes_per_launch": corrected}
open(os.path.join(dst, f"{rnd}_pmc_summary.csv"), "w").write("\n".join(lines) + "\n")
k = out.get("k_iso_work")
json.dump({"kernel": "k_iso_work", "bytes_per_launch": k["bytes_per_launch"] if k else None,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) on bench.py; "
                     "FETCH_SIZE x2 (gfx950 correction), KiB -> bytes", "per_kernel": out},
          open(os.path.join(dst, f"traffic_{rnd}.json"), "w"), indent=1)
print("\n".join(lines))
