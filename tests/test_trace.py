"""Trace mode (qkd_trace_decode / qkd_ldpc_amd.trace_decode): the reference's
TRACE_SUM_PRODUCT ("E:", "L:", "z:", "s:", "M:") and TRACE_SUM_PRODUCT_LLR
(MAX_LLR) output of one frame (qkd_ldpc_algorithm.cpp:212-330), decoded on the
device. Checked against the reference's own recorded textbook traces
(tests/golden/reference_probe.json) and, per iteration and bit for bit,
against the oracle's message trace.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def Q():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import qkd_ldpc_amd as Q
    return Q


def sig(x, digits):
    return float(f"{x:.{digits}g}")


def test_textbook_n10_trace_matches_reference(Q, probe):
    p = probe["textbook_n10"]
    dense = np.array(p["dense"], np.uint8)
    H = Q.HMatrix.from_dense_array(dense)
    q = p["qber"]
    lp = np.log((1 - q) / q)
    llr = np.where(np.array(p["bob"]) == 1, -lp, lp)
    syn = dense.astype(int) @ np.array(p["alice"]) % 2
    tr = Q.trace_decode(H, llr, syn, p["max_it"], p["thr"], True)
    assert tr["iterations"] == p["iterations"] and tr["syndromes_match"]
    assert [sig(x, 4) for x in tr["L"][0]] == p["L_iter1_4sig"]
    assert tr["max_llr"] == p["max_llr"]                    # 17 significant digits
    assert (tr["s"][-1] == np.array(p["alice_syndrome"])).all()
    assert (tr["z"][-1] == np.array(p["alice"])).all()


def test_textbook_n6_trace_matches_reference(Q, probe):
    p = probe["textbook_n6"]
    dense = np.array(p["dense"], np.uint8)
    H = Q.HMatrix.from_dense_array(dense)
    q = p["qber"]
    lp = np.log((1 - q) / q)
    llr = np.where(np.array(p["bob"]) == 1, -lp, lp)
    syn = dense.astype(int) @ np.array(p["alice"]) % 2
    tr = Q.trace_decode(H, llr, syn, p["max_it"], p["thr"], True)
    assert tr["iterations"] == 1 and tr["syndromes_match"]
    cptr, cidx, bptr, bidx = H.adjacency()
    assert [round(float(x), 4) for x in tr["E"][0][bptr[0]:bptr[1]]] == p["first_c2b_row_4dp"]
    assert [sig(x, 4) for x in tr["L"][0]] == p["L_iter1_4sig"]
    assert tr["M"].shape[0] == 0 and tr["max_llr"] == 0.0     # stopped at once: no M, MAX_LLR 0


@pytest.mark.parametrize("q,thr,thr_on,max_it", [(0.05, 100.0, True, 50), (0.08, 2.5, True, 30),
                                                 (0.06, 0.0, False, 50), (0.09, 100.0, True, 4)])
def test_trace_equals_oracle_per_iteration(Q, golden_code, oracle_mod, oracle_code, q, thr, thr_on, max_it):
    H = Q.HMatrix.from_check_lists(int(golden_code["dims"][0]), golden_code["chk_off"], golden_code["chk_idx"])
    s = int(oracle_mod.seeds(4321, 1)[0])
    a, b, qq = oracle_mod.keygen(s, 10240, q)
    lp = np.log((1 - qq) / qq)
    llr = np.where(b == 1, -lp, lp)
    syn = oracle_code.syndrome(a)
    want = oracle_code.decode(llr, syn, max_it, thr, thr_on, ltrace=True, etrace=True)
    tr = Q.trace_decode(H, llr, syn, max_it, thr if thr_on else 100.0, thr_on)
    assert tr["iterations"] == want["iters"] and tr["syndromes_match"] == want["sp_ok"]
    assert tr["E"].shape == want["etrace"].shape
    assert (tr["E"].view(np.uint64) == want["etrace"].view(np.uint64)).all()     # bit patterns
    assert (tr["L"].view(np.uint64) == want["ltrace"].view(np.uint64)).all()
    assert (tr["z"][-1] == want["out"]).all()
    assert tr["max_llr"] == want["max_llr"]


def test_trace_rejects_variants(Q, golden_code):
    H = Q.HMatrix.from_check_lists(int(golden_code["dims"][0]), golden_code["chk_off"], golden_code["chk_idx"])
    from qkd_ldpc_amd import _native as N
    llr = np.ones(10240)
    syn = np.zeros(H.num_check_nodes, np.uint8)
    it = np.zeros(1, np.uint32)
    ok = np.zeros(1, np.uint8)
    st = N.lib().qkd_trace_decode(H.handle, llr.ctypes.data, syn.ctypes.data, 5, 100.0,
                                  Q.decoder_flags(True, "minsum"), None, None, it.ctypes.data, ok.ctypes.data)
    assert st == N.ERR_UNSUPPORTED if hasattr(N, "ERR_UNSUPPORTED") else st == 8
