"""Attribute kernels to the library calls that launched them, from a rocprofv3 run with
--kernel-trace --marker-trace --hip-runtime-trace (tools/prof_roctx.sh; GRAPHBLAS_AMD_ROCTX=1
makes every GrB_* / GxB_* entry point push a roctx range named after itself).  A kernel's
correlation id names the HIP launch call that enqueued it; the kernel belongs to the innermost
roctx range open on that call's thread at that host time.  Prints, per entry point: ranges,
kernels launched and the GPU time of those kernels (the kernel-level view of the reference's
Recorder, core/recorder.py:34-178)."""
import bisect
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]


def load(pat):
    f = sorted(glob.glob(os.path.join(d, pat)))
    return list(csv.DictReader(open(f[0]))) if f else []


kern = load("*kernel_trace.csv")
mark = load("*marker_api_trace.csv")
api = load("*hip_api_trace.csv")
if not mark:
    print("no marker trace; files:", os.listdir(d))
    sys.exit(0)
cols = list(mark[0].keys())
msgk = next((c for c in ("Message", "Marker_Message", "Name", "Function") if c in cols), None)
# ranges per thread, as (start, end, name); nesting resolved by taking the innermost (latest start)
ranges = collections.defaultdict(list)
for r in mark:
    try:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    except (KeyError, ValueError):
        continue
    if e > s and r.get(msgk):
        ranges[r.get("Thread_Id")].append((s, e, r[msgk]))
for t in ranges:
    ranges[t].sort()
starts = {t: [x[0] for x in v] for t, v in ranges.items()}
launch = {r["Correlation_Id"]: (int(r["Start_Timestamp"]), r.get("Thread_Id")) for r in api}


def owner(ts, tid):
    v = ranges.get(tid)
    if not v:
        return None
    i = bisect.bisect_right(starts[tid], ts) - 1
    while i >= 0:  # innermost open range: the latest-starting one that has not ended
        s, e, n = v[i]
        if e >= ts:
            return n
        i -= 1
    return None


stat = collections.defaultdict(lambda: [0, 0.0])
nr = collections.Counter(n for v in ranges.values() for _, _, n in v)
miss = 0
for k in kern:
    c = launch.get(k["Correlation_Id"])
    n = owner(*c) if c else None
    if n is None:
        miss += 1
        n = "(outside any library call)"
    stat[n][0] += 1
    stat[n][1] += (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
print(f"{'entry point':44s} {'ranges':>8s} {'kernels':>8s} {'GPU us':>12s}")
for n, (nk, us) in sorted(stat.items(), key=lambda kv: -kv[1][1]):
    print(f"{n[:44]:44s} {nr.get(n, 0):8d} {nk:8d} {us:12.1f}")
print(f"marker columns: {cols}; kernels without a launching range: {miss} of {len(kern)}")
