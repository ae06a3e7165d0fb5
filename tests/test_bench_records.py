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


def test_stale_record_is_never_traffic(tmp_path):
    """A PMC record without a source hash, or with one that differs from the tree's
    sources of its kernel, is marked stale and gives no ``traffic``."""
    kernel = "regrid_coarsen_cells_kernel"
    fresh = bench.kernel_source_hash(kernel)
    assert fresh and len(fresh) == 16
    assert "mappm_core.h" in bench.kernel_sources(kernel) and "mappm_multi.h" in bench.kernel_sources(kernel)
    recs = {"old": {"kernel": kernel, "hbm_bytes_per_launch": 1.0, "profile": "r04y"},
            "moved": {"kernel": kernel, "hbm_bytes_per_launch": 1.0, "profile": "r05", "src_hash": "0" * 16},
            "fresh": {"kernel": kernel, "hbm_bytes_per_launch": 2.0, "profile": "r06", "src_hash": fresh}}
    path = tmp_path / "pmc.json"
    path.write_text(json.dumps(recs))
    assert bench.pmc_record("old", str(path))["stale"]
    assert bench.pmc_record("moved", str(path))["stale"]
    assert not bench.pmc_record("fresh", str(path))["stale"]


def test_with_counters_drops_stale_traffic(monkeypatch):
    monkeypatch.setattr(bench, "pmc_record", lambda leg: {"kernel": "dense_forward_kernel", "stale": True,
                                                        "hbm_bytes_per_launch": 5.0, "profile": "r03c"})
    rec = bench.with_counters("dense_c48", {}, alg_bytes=1.0)
    assert rec["traffic"] is None and rec["pmc_stale"]["profile"] == "r03c"
    assert bench.compact_leg(rec)["pmc"] == "r03c (stale)"


def _recorded_result():
    """The round-5 closing bench run's verbose line (every leg, profiles/bench_r05zzn.json)."""
    with open(os.path.join(ROOT, "profiles", "bench_r05zzn.json")) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_compact_line_fits_driver_budget():
    """The driver keeps ~8 KB of stdout and parses the last line: the line carries the
    contract fields, roofline and cpu_baseline, and a terse summary of every leg, in at
    most bench.LINE_BUDGET characters."""
    full = _recorded_result()
    assert len(json.dumps(full)) > bench.LINE_BUDGET  # the round-5 line that did not parse
    line = bench.compact_line(full)
    assert len(line) <= bench.LINE_BUDGET
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "higher_is_better", "scaling", "vs_baseline"):
        assert k in d, k
    assert d["roofline"]["frac"] > 0 and d["cpu_baseline"]["value"] > 0
    assert set(d["extra"]) == set(full["extra"]) and set(d["extra_scaling"]) == set(full["extra_scaling"])
    for leg in d["extra"].values():
        assert "ms" in leg
    assert d["extra"]["stepper_c96_rank_of_8"]["ratio"] > 0


def test_leg_recorder_keeps_finished_legs(tmp_path):
    """Every assignment is on disk at once; a later re-assignment of a leg wins."""
    path = str(tmp_path / "legs.jsonl")
    rec = bench.LegRecorder(path)
    rec["a"] = {"ms_per_step": 1.0}
    rec["scaling/b"] = {"ms_per_step": 2.0}
    rec["a"] = dict(rec["a"], cpu_baseline={"value": 3.0})
    legs = {}
    with open(path) as f:
        for ln in f:
            legs.update(json.loads(ln))
    assert legs == {"a": {"ms_per_step": 1.0, "cpu_baseline": {"value": 3.0}}, "scaling/b": {"ms_per_step": 2.0}}
