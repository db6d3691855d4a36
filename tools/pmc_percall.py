"""Turn a tools/pmc_table.py table (gpurun_out/<name>_table.json) into a committed per-call
profile (profiles/<out>.json): the table plus `calls`, the command it came from, and
hbm_bytes_per_call = sum over the per-call kernels of hbm_bytes_per_launch x launches / calls
(kernels launched fewer times than there are calls -- input generation, the matrix's cached
tables built on first use -- are one-time setup, listed apart and left out).
bench.py reads hbm_bytes_per_call as a secondary line's roofline `traffic`.
usage: python3 tools/pmc_percall.py NAME OUT CALLS "command description" """
import json
import os
import sys

name, out, calls, cmd = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
t = json.load(open(os.path.join(root, "gpurun_out", f"{name}_table.json")))
tot = 0.0
per_kernel, once = {}, {}
for k, v in t["kernels"].items():
    if "hbm_bytes_per_launch" in v and v.get("launches"):
        if v["launches"] < calls:
            once[k] = v["hbm_bytes_per_launch"] * v["launches"]
            continue
        b = v["hbm_bytes_per_launch"] * v["launches"] / calls
        per_kernel[k] = b
        tot += b
t["calls"] = calls
t["command"] = cmd
t["hbm_bytes_per_call"] = tot
t["hbm_bytes_per_call_by_kernel"] = dict(sorted(per_kernel.items(), key=lambda kv: -kv[1]))
t["one_time_hbm_bytes_by_kernel"] = once
json.dump(t, open(os.path.join(root, "profiles", f"{out}.json"), "w"), indent=1)
print(f"{out}: {tot / 1e9:.2f} GB per call over {calls} calls")
for k, b in list(t["hbm_bytes_per_call_by_kernel"].items())[:8]:
    print(f"  {b / 1e9:8.2f} GB  {k[:90]}")
