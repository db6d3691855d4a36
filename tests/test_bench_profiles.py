"""Measurement hygiene: every roofline `traffic` the bench reports comes from a
committed profile of this round, and the bench prefers that round's files.  CPU only: reads the
committed JSON profiles and bench.py's lookup, runs nothing on a GPU."""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (module level: argparse, numpy, scipy only)

# the newest round with a committed headline traffic file: its profiles must be complete
ROUND = bench.CUR_ROUND

# the per-call profiles the secondary lines read (bench.py config2_spmv / config4_masked_spgemm /
# config5_spgemm)
SECONDARY = [
    "config2_s22_pmc.json",
    "config2_s22_ef60_pmc.json",
    "config4_s20_pmc.json",
    "config4_s22_pmc.json",
    "config5_s19_pmc.json",
    "config5_s20_pmc.json",
]


def test_round_is_the_newest_profile_round():
    import glob
    rounds = [int(os.path.basename(f)[len("traffic_r"):-len(".json")])
              for f in glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json"))]
    assert rounds and ROUND == f"r{max(rounds):02d}"


@pytest.mark.parametrize("stem", SECONDARY)
def test_secondary_traffic_from_this_round(stem):
    name = f"{ROUND}_{stem}"
    traffic, src = bench._profile_traffic(stem)
    assert src == f"profiles/{name}", f"{name} missing from profiles/"
    assert traffic and traffic > 0
    d = json.load(open(os.path.join(ROOT, src)))
    assert d["calls"] >= 1 and d["command"]
    assert d["hbm_bytes_per_call_by_kernel"], "per-kernel split of the call's bytes"


def test_bench_prefers_this_rounds_profiles():
    """bench.py's lookups carry no hard-coded round: the newest round is tried first"""
    src = open(os.path.join(ROOT, "bench.py")).read()
    calls = re.findall(r"_profile_traffic\(\s*f?\"([a-z0-9_{}.]+)", src)
    assert len(calls) >= 3, calls
    for first in calls:
        assert not re.match(r"r\d+_", first), first
    assert bench.ROUNDS[0] == ROUND


def test_headline_traffic_file():
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'f"traffic_{CUR_ROUND}.json"' in src
    t = json.load(open(os.path.join(ROOT, "profiles", f"traffic_{ROUND}.json")))
    assert t["kernel"] == "k_iso_work"
    # PMC bytes per launch of the headline kernel vs SURVEY 8(d)'s 43.3 MB algorithmic at s22:
    # a committed profile of the real workload, not a placeholder
    assert 40e6 < t["bytes_per_launch"] < 60e6
