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


def mix_priced_frac(c):
    """Recomputed from the committed files, independently of bench.py and
    tools/pmc_traffic.py: the dynamic opcode census (profiles/r*_valu_census.json,
    tools/valu_census.py's classes and measured-opcode aliases) weights each
    opcode's 4-wave issue cost (profiles/r*_issue_mb.txt) into one price per PMC
    class; each class of the PMC record (OTHER = SQ_INSTS_VALU minus the classed
    ones) at its price, over the kernel's SIMD-cycles."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import valu_census as V
    census = json.load(open(newest("r*_valu_census.json")))["dynamic_per_launch"]
    costs = V.load_costs(newest("r*_issue_mb.txt"))
    num, den = {}, {}
    for op, n in census.items():
        cyc, _ = V.opcode_cost(op, costs)
        if cyc is None:
            continue
        k = V.pmc_class(op)
        num[k] = num.get(k, 0.0) + n * cyc
        den[k] = den.get(k, 0.0) + n
    mean = sum(num.values()) / sum(den.values())
    price = {k: num[k] / den[k] for k in num}
    g = lambda n: c.get("SQ_INSTS_VALU_" + n, 0.0)
    cls = {"FMA_F32": g("FMA_F32"), "MUL_F32": g("MUL_F32"), "ADD_F32": g("ADD_F32"), "TRANS_F32": g("TRANS_F32"),
           "F64": g("ADD_F64") + g("MUL_F64") + g("FMA_F64"), "TRANS_F64": g("TRANS_F64"), "INT32": g("INT32"),
           "INT64": g("INT64"), "CVT": g("CVT")}
    cls["OTHER"] = c["SQ_INSTS_VALU"] - sum(cls.values())
    assert cls["OTHER"] >= 0
    price.setdefault("TRANS_F64", 2 * costs["v_fma_f64"])
    need = sum(n * price.get(k, mean) for k, n in cls.items())
    return need / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)


def test_census_prices_every_hot_opcode():
    """The census's opcodes are priced by measured ones: at least 99 % of its
    dynamic VALU count, and OTHER's price is the census-weighted mean, not a
    fixed mean of a few opcodes."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import valu_census as V
    census = json.load(open(newest("r*_valu_census.json")))["dynamic_per_launch"]
    costs = V.load_costs(newest("r*_issue_mb.txt"))
    tot = sum(census.values())
    priced = sum(n for op, n in census.items() if V.opcode_cost(op, costs)[0] is not None)
    assert priced / tot >= 0.99
    other = {op: n for op, n in census.items() if V.pmc_class(op) == "OTHER"}
    assert sum(other.values()) / tot > 0.3          # (the selects, moves and shifts the verdict asked about)


def test_headline_roofline_is_valu_issue_from_the_pmc_record():
    import bench
    rec = json.load(open(newest("r*_pmc_sp_f64.json")))
    v = rec["valu"]
    alg = 12905 * bench.B_ITER + 4096 * bench.B_FRAME          # config 2
    rb = bench.roofline_block("sp_f64", alg, 1.45e-3, 1.55e-3, "decoder")
    c = rec["counters"]
    simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
    want_2cyc = c["SQ_INSTS_VALU"] * 2 / simd_cycles
    assert rb["bound"] == "valu"
    assert abs(rb["frac_2cyc"] - want_2cyc) < 1e-12 and 0 < want_2cyc <= 1
    if "SQ_INSTS_VALU_FMA_F32" in c:
        assert abs(rb["frac"] - mix_priced_frac(c)) < 1e-9
    else:                                     # a record without the VALU class passes
        assert abs(rb["frac"] - want_2cyc) < 1e-12
    assert 0 < rb["frac"] <= 1
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
