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


def issue_4waves():
    """4 waves/SIMD, ILP 8 rows of the committed issue micro-benchmark."""
    cost = {}
    for line in open(os.path.join(ROOT, "profiles", "r05_issue_mb.txt")):
        f = line.split()
        if f[2] == "4.0" and f[4] == "8":
            cost[f[0]] = float(f[-1])
    return cost


def mix_priced_frac(c):
    """Restated independently of tools/pmc_traffic.py: each VALU class of the PMC
    record at its measured 4-wave issue cost (binary32 FMA / MUL / ADD split packed
    vs scalar by the census shares DESIGN.md §4.3 states; the unclassified rest at
    the mean of v_mov, v_xor, v_bfe, v_med3, v_cmp, v_cndmask with an SGPR mask),
    over the kernel's SIMD-cycles."""
    k = issue_4waves()
    pk = {"FMA": (0.62, "v_pk_fma_f32", "v_fma_f32"), "MUL": (0.45, "v_pk_mul_f32", "v_mul_f32"),
          "ADD": (0.63, "v_pk_add_f32", "v_add_f32")}
    g = lambda n: c.get("SQ_INSTS_VALU_" + n, 0.0)
    need, counted = 0.0, 0.0
    for cls, (share, p, q) in pk.items():
        need += g(cls + "_F32") * (share * k[p] + (1 - share) * k[q])
        counted += g(cls + "_F32")
    trans = (k["v_exp_f32"] + k["v_log_f32"] + k["v_rcp_f32"]) / 3
    f64 = g("ADD_F64") + g("MUL_F64") + g("FMA_F64")
    need += g("TRANS_F32") * trans + f64 * k["v_fma_f64"] + g("TRANS_F64") * 2 * k["v_fma_f64"]
    need += (g("INT32") + g("CVT")) * k["v_add_u32"] + g("INT64") * 2 * k["v_add_u32"]
    counted += g("TRANS_F32") + f64 + g("TRANS_F64") + g("INT32") + g("CVT") + g("INT64")
    kinds = ("v_mov_b32", "v_xor_b32", "v_bfe_u32", "v_med3_f32", "v_cmp_gt_f32", "v_cndmask_b32_sgpr")
    rest = sum(k[x] for x in kinds) / len(kinds)
    need += max(0.0, c["SQ_INSTS_VALU"] - counted) * rest
    return need / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)


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
