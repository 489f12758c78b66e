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


def test_valu_mix_prices_the_counts_at_the_issue_table():
    import pmc_traffic as T
    cost = T.issue_costs()
    for k in ("v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_cndmask_b32_sgpr", "v_add_u32"):
        assert k in cost and cost[k] > 0
    c = {"SQ_INSTS_VALU": 1000.0, "SQ_INSTS_VALU_FMA_F32": 100.0, "SQ_INSTS_VALU_MUL_F32": 50.0,
         "SQ_INSTS_VALU_ADD_F32": 50.0, "SQ_INSTS_VALU_TRANS_F32": 20.0, "SQ_INSTS_VALU_INT32": 80.0,
         "SQ_INSTS_VALU_INT64": 10.0}
    cycles = 100.0                                     # per XCD-averaged GPU cycle count
    m = T.valu_mix(c, cycles)
    s = T.PACKED_SHARE
    want = (100 * (s["FMA_F32"] * cost["v_pk_fma_f32"] + (1 - s["FMA_F32"]) * cost["v_fma_f32"])
            + 50 * (s["MUL_F32"] * cost["v_pk_mul_f32"] + (1 - s["MUL_F32"]) * cost["v_mul_f32"])
            + 50 * (s["ADD_F32"] * cost["v_pk_add_f32"] + (1 - s["ADD_F32"]) * cost["v_add_f32"])
            + 20 * (cost["v_exp_f32"] + cost["v_log_f32"] + cost["v_rcp_f32"]) / 3
            + 80 * cost["v_add_u32"] + 10 * 2 * cost["v_add_u32"]
            + (1000 - 310) * sum(cost[k] for k in T.OTHER_KINDS) / len(T.OTHER_KINDS))
    assert m["simd_cycles_needed"] == pytest.approx(want, rel=1e-12)
    assert m["frac_mix"] == pytest.approx(want / (cycles * 1024), rel=1e-12)
    assert m["counts"]["OTHER"] == 690.0
    # a record without the class counters has no mix
    assert T.valu_mix({"SQ_INSTS_VALU": 1.0}, cycles) is None
