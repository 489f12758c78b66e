"""The profiling tools behind profiles/r05_* (CPU): the phase-stop patch applies
to the shipped decoder source exactly once per anchor, and the VALU-mix pricing
of tools/pmc_traffic.py reads the committed issue table and prices a synthetic
record by hand."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_phase_stop_patch_applies_to_the_decoder():
    import phase_stop_patch as P
    src = open(os.path.join(ROOT, "qkd_ldpc_amd", "csrc", "decode_split.hip")).read()
    out = P.patch(src)
    # one stop point after each check phase, bit phase and syndrome test, one at the loop top
    assert out.count("QKD_STOP_POINT") == 3 + 1          # three uses + the macro definition
    assert "QKD_PMC_STOP == 0) break;" in out
    assert out.count("uint32_t pmc_ph = 0;") == 1
    # the product source itself carries no stop points
    assert "QKD_STOP_POINT" not in src


def test_valu_mix_prices_the_counts_at_the_census_weighted_costs(tmp_path):
    """A synthetic census (two OTHER opcodes, a packed and a scalar FMA) and a
    synthetic record: each class at its census-weighted issue cost."""
    import json
    import pmc_traffic as T
    import valu_census as V
    cost = V.load_costs(os.path.join(ROOT, "profiles", "r06_issue_mb.txt"))
    for k in ("v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_cndmask_b32_sgpr", "v_add_u32", "v_lshrrev_b32"):
        assert k in cost and cost[k] > 0
    census = {"v_cndmask_b32": 30.0, "v_lshrrev_b32": 10.0, "v_pk_fma_f32": 3.0, "v_fma_f32": 1.0,
              "v_add_u32": 5.0, "v_exp_f32": 2.0}
    p = tmp_path / "census.json"
    p.write_text(json.dumps({"dynamic_per_launch": census}))
    c = {"SQ_INSTS_VALU": 1000.0, "SQ_INSTS_VALU_FMA_F32": 100.0, "SQ_INSTS_VALU_TRANS_F32": 20.0,
         "SQ_INSTS_VALU_INT32": 80.0}
    cycles = 100.0                                     # per XCD-averaged GPU cycle count
    m = T.valu_mix(c, cycles, census_path=str(p), issue_path=os.path.join(ROOT, "profiles", "r06_issue_mb.txt"))
    other = (30 * cost["v_cndmask_b32_sgpr"] + 10 * cost["v_lshrrev_b32"]) / 40
    fma = (3 * cost["v_pk_fma_f32"] + 1 * cost["v_fma_f32"]) / 4
    want = 100 * fma + 20 * cost["v_exp_f32"] + 80 * cost["v_add_u32"] + (1000 - 200) * other
    assert m["simd_cycles_needed"] == pytest.approx(want, rel=1e-12)
    assert m["frac_mix"] == pytest.approx(want / (cycles * 1024), rel=1e-12)
    assert m["counts"]["OTHER"] == 800.0
    # a record without the VALU total has no mix
    assert T.valu_mix({"SQ_X": 1.0}, cycles) is None
