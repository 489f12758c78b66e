"""bench.py's roofline block (CPU): bound by the VALU issue rate of the committed PMC
record, a fraction <= 1 reproducible from that file alone, with SURVEY.md §8(d)'s
algorithmic bytes kept only as the nominal figure."""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def newest(pattern):
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        pytest.skip(f"no profiles/{pattern}")
    return files[-1]


def test_headline_roofline_is_valu_issue_from_the_pmc_record():
    import bench
    rec = json.load(open(newest("r*_pmc_sp_f64.json")))
    v = rec["valu"]
    alg = 12905 * bench.B_ITER + 4096 * bench.B_FRAME          # config 2
    rb = bench.roofline_block("sp_f64", alg, 1.45e-3, 1.55e-3, "decoder")
    want = rec["counters"]["SQ_INSTS_VALU"] * 2 / (rec["counters"]["GRBM_GUI_ACTIVE"] / 8 * 1024)
    assert rb["bound"] == "valu"
    assert abs(rb["frac"] - want) < 1e-12 and 0 < rb["frac"] <= 1
    assert abs(rb["achieved"] / rb["peak"] - rb["frac"]) < 1e-12
    assert rb["traffic"] == rec["hbm_bytes_per_launch"]
    # the nominal HBM figure: algorithmic bytes over the live kernel time, no longer the headline
    assert abs(rb["nominal_frac"] - alg / 1.45e-3 / 8e12) < 1e-12
    assert rb["nominal_frac"] > 1 and "not an achieved bandwidth" in rb["nominal_note"]
    assert 0 < rb["hbm_frac_measured"] < 1
    assert abs(rb["live"]["frac_at_rated_clock"] - v["valu_insts_per_launch"] * 2 / (1.45e-3 * 2.4e9 * 1024)) < 1e-12


def test_roofline_without_a_pmc_record_is_marked_nominal(monkeypatch):
    import bench
    monkeypatch.setattr(bench, "pmc_record", lambda variant: (None, None))
    rb = bench.roofline_block("sp_f64", 1e9, 1e-3, 1e-3, "decoder")
    assert rb["bound"] == "hbm" and rb["nominal"] is True and rb["traffic"] is None
