"""bench.py's record helpers on the committed PMC evidence (CPU only: no kernel runs).

Every leg in profiles/pmc_traffic.json must turn into a bench record without error, and
the VALU issue fraction must follow from the committed counters and the measured issue
peaks (profiles/valu_calib.json), never above 1."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
    LEGS = sorted(json.load(f))


@pytest.mark.parametrize("leg", LEGS)
def test_with_counters_builds_every_leg(leg):
    rec = bench.with_counters(leg, {}, alg_bytes=1.0)
    assert "traffic" in rec
    if "valu_issue_frac" in rec:
        assert 0.0 < rec["valu_issue_frac"] <= 1.0
        if "valu_issue_frac_lo" in rec:
            assert rec["valu_issue_frac_lo"] <= rec["valu_issue_frac"]


def test_unknown_leg_has_no_traffic():
    assert bench.with_counters("no_such_leg", {}) == {"traffic": None}
