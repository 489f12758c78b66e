"""The oracle (oracle/oracle.c) pinned against the reference's recorded outputs
(tests/golden/reference_probe.json) and the committed
golden vectors regenerated from it."""
import os

import numpy as np
import pytest

from tests.conftest import REF_ROOT


def test_seeds_match_reference(probe, oracle_mod):
    s = oracle_mod.seeds(777, 4)
    assert int(s[0]) == int(probe["seeds_777_first"])


@pytest.mark.parametrize("case", ["textbook_n6", "textbook_n10"])
def test_textbook_known_answers(probe, oracle_mod, case):
    p = probe[case]
    code = oracle_mod.Code.from_dense(np.array(p["dense"], np.uint8))
    alice = np.array(p["alice"])
    bob = np.array(p["bob"])
    q = p["qber"]
    lp = np.log((1 - q) / q)
    llr = np.where(bob == 1, -lp, lp)
    syn = code.syndrome(alice)
    if "alice_syndrome" in p:
        assert syn.tolist() == p["alice_syndrome"]
    r = code.decode(llr, syn, p["max_it"], p["thr"], True, ltrace=True)
    assert r["iters"] == p["iterations"]
    assert r["sp_ok"] == p["syndromes_match"]
    assert (r["out"] == alice).all() == p["keys_match"]
    L1 = r["ltrace"][0]
    for got, want in zip(L1, p["L_iter1_4sig"]):
        assert float(f"{got:.4g}") == want
    if "max_llr" in p:
        assert r["max_llr"] == p["max_llr"]          # 17 significant digits
    q2 = code.qkd_ldpc(alice, bob, q, p["max_it"], p["thr"], True)
    assert q2["key_ok"] == p["keys_match"] and q2["iters"] == p["iterations"]


def test_config2_frame0(probe, oracle_code, oracle_mod):
    p = probe["config2_frame0"]
    a, b, q = oracle_mod.keygen(int(p["seed"]), 10240, p["qber_nominal"])
    assert int((a != b).sum()) == p["errors"]
    r = oracle_code.run_trial(p["qber_nominal"], int(p["seed"]))
    assert r["iters"] == p["iterations"] and r["sp_ok"] == p["success"] and r["key_ok"]


def test_config2_aggregates(probe, oracle_code, oracle_mod):
    p = probe["config2"]
    seeds = oracle_mod.seeds(p["simulation_seed"], p["trials"])
    r = oracle_code.trials(p["qber_nominal"], seeds, 0, p["max_it"], p["thr"], True,
                           threads=min(8, os.cpu_count() or 1))
    st = oracle_mod.batch_stats(r["iters"], r["sp_ok"], r["key_ok"], r["exact_q"], p["trials"],
                                p["max_it"])
    assert st["sum_iters_sp"] == p["sum_iterations"]
    assert float(f"{st['iterations_successful_sp_mean']:.6g}") == p["mean_6sig"]
    assert float(f"{st['iterations_successful_sp_std_dev']:.6g}") == p["std_6sig"]
    assert (st["iterations_successful_sp_min"], st["iterations_successful_sp_max"]) == (p["min"], p["max"])
    assert st["fer"] == p["fer"]


def test_golden_vectors_reproduce_reference_tables(probe, golden_vectors, oracle_mod):
    """config-2/3 per-frame fixtures reduce to the reference's published aggregates."""
    g = golden_vectors
    st = oracle_mod.batch_stats(g["c2_iters"], g["c2_sp"], g["c2_ko"], np.repeat(g["c2_q"], 2),
                                4096, 50)
    assert st["sum_iters_sp"] == probe["config2"]["sum_iterations"]
    for s, pp in enumerate(probe["config3"]["points"]):
        st = oracle_mod.batch_stats(g["c3_iters"][s], g["c3_sp"][s], g["c3_ko"][s], g["c3_q"][s:s + 1],
                                    10000, 50)
        assert round(st["initial_QBER"], 5) == round(pp["qber_actual"], 5)
        assert abs(st["iterations_successful_sp_mean"] - pp["mean_it"]) <= 5e-4 + 1e-9
        assert abs(st["fer"] - pp["fer"]) < 1e-12


def test_golden_vectors_regenerate(golden_vectors, oracle_code, oracle_mod):
    """A sample of the committed per-frame fixtures, recomputed by the oracle now."""
    g = golden_vectors
    seeds = oracle_mod.seeds(777, 10000)
    r = oracle_code.trials(0.02, seeds[:256], 0, 50, 100.0, True)
    assert (r["iters"] == g["c2_iters"][:256]).all()
    pick = np.arange(0, 10000, 997)
    r = oracle_code.trials(float(g["c3_qnom"][7]), seeds[pick], 7, 50, 100.0, True)
    assert (r["iters"] == g["c3_iters"][7][pick]).all()
    assert (r["key_ok"] == g["c3_ko"][7][pick]).all()
    k = len(g["kg_seeds"])
    for idx in (0, k + 3, 2 * k + 5, 3 * k + 1):
        a, b, q = oracle_mod.keygen(int(g["kg_seeds"][idx % k]), 10240, float(g["kg_qnom"][idx]))
        assert (np.packbits(a.astype(np.uint8)) == g["kg_alice"][idx]).all()
        assert (np.packbits(b.astype(np.uint8)) == g["kg_bob"][idx]).all()
        assert q == g["kg_q"][idx]


def test_golden_code_matches_reference_file(golden_code, oracle_mod):
    path = os.path.join(REF_ROOT, "alist_sparse_matrices", "(N=10240,M=5231,R=0.49,CW=3,SEED=666).txt")
    if not os.path.exists(path):
        pytest.skip("reference tree not present (GPU box)")
    code = oracle_mod.Code.from_alist(path)
    bo, bi, co, ci = code.lists()
    assert (bo == golden_code["bit_off"]).all() and (bi == golden_code["bit_idx"]).all()
    assert (co == golden_code["chk_off"]).all() and (ci == golden_code["chk_idx"]).all()


def test_adjacency_sorted_and_consistent(golden_code):
    """Invariant A1: every row ascending, both lists the same edge set."""
    g = golden_code
    for off, idx in ((g["bit_off"], g["bit_idx"]), (g["chk_off"], g["chk_idx"])):
        for r in range(off.size - 1):
            row = idx[off[r]:off[r + 1]]
            assert (np.diff(row) > 0).all()
    edges_b = {(int(c), i) for i in range(10240) for c in g["bit_idx"][g["bit_off"][i]:g["bit_off"][i + 1]]}
    edges_c = {(j, int(b)) for j in range(5231) for b in g["chk_idx"][g["chk_off"][j]:g["chk_off"][j + 1]]}
    assert edges_b == edges_c and len(edges_b) == 30720
