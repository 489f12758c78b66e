"""The C++ compatibility shim (compat/): the reference's own signatures
(qkd_ldpc_algorithm.hpp, array_and_matrix_operations.hpp:39-40, simulation.hpp:49-50)
on top of the C ABI, driven the way the reference's callers drive them.

CPU: the shim library builds, exports every reference symbol, and the driver links.
GPU: results equal the oracle (decoded words, iterations, flags, run_trial, and the
QKD_LDPC_batch_simulation statistics of simulation.cpp:252-312 to the last bit)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "qkd_ldpc_amd", "lib")

REFERENCE_SYMBOLS = [
    "sum_product_decoding_regular(double const*, H_matrix const&, int const*, unsigned long const&, double const&, int*)",
    "sum_product_decoding_irregular(double const*, H_matrix const&, int const*, unsigned long const&, double const&, int*)",
    "QKD_LDPC_regular(int const*, int const*, double const&, H_matrix const&)",
    "QKD_LDPC_irregular(int const*, int const*, double const&, H_matrix const&)",
    "calculate_syndrome_regular(int const*, H_matrix const&, int*)",
    "calculate_syndrome_irregular(int const*, H_matrix const&, int*)",
    "run_trial(H_matrix const&, double, unsigned long)",
    "QKD_LDPC_batch_simulation(std::vector<sim_input, std::allocator<sim_input> > const&)",
]


@pytest.fixture(scope="module")
def compat_lib():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "compat")])
    return os.path.join(LIB, "libqkd_ldpc_compat.so")


@pytest.fixture(scope="module")
def driver(compat_lib, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("compat") / "compat_driver")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", out,
                           os.path.join(ROOT, "tests", "native", "compat_driver.cpp"),
                           f"-L{LIB}", "-lqkd_ldpc_compat", "-lqkd_ldpc_amd", f"-Wl,-rpath,{LIB}"])
    return out


def test_compat_exports_reference_symbols(compat_lib):
    out = subprocess.check_output(["nm", "-DC", "--defined-only", compat_lib], text=True)
    for sym in REFERENCE_SYMBOLS:
        assert sym in out, sym


def test_compat_driver_links(driver):
    assert os.path.exists(driver)


# ---- GPU ----------------------------------------------------------------------------

def _code_cmd(n, m, chk_off, chk_idx):
    lines = [f"code {n} {m}"]
    for j in range(m):
        row = chk_idx[chk_off[j]:chk_off[j + 1]]
        lines.append(f"{len(row)} " + " ".join(str(int(x)) for x in row))
    return lines


def _run(driver, lines):
    p = subprocess.run([driver], input="\n".join(lines) + "\n", text=True, capture_output=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr
    out = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert not any(ln.startswith(("exception", "error")) for ln in out), out
    return out


def _dense_lists(dense):
    off, idx = [0], []
    for row in dense:
        idx.extend(np.nonzero(row)[0].tolist())
        off.append(len(idx))
    return np.array(off), np.array(idx)


def _fmt(v):
    return " ".join(repr(float(x)) if isinstance(x, (float, np.floating)) else str(int(x)) for x in v)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["textbook_n6", "textbook_n10"])
def test_compat_textbook_example(driver, probe, oracle_mod, case):
    """BASELINE config 1: example/qkd_ldpc_example.cpp's flow through the shim."""
    p = probe[case]
    dense = np.array(p["dense"], np.uint8)
    off, idx = _dense_lists(dense)
    oc = oracle_mod.Code.from_dense(dense)
    n, m = dense.shape[1], dense.shape[0]
    alice, bob, q = np.array(p["alice"]), np.array(p["bob"]), p["qber"]
    lp = np.log((1 - q) / q)
    llr = np.where(bob == 1, -lp, lp)
    syn = oc.syndrome(alice)
    out = _run(driver, _code_cmd(n, m, off, idx) + [
        f"cfg {p['max_it']} {p['thr']!r} 1 1 777",
        "decode", _fmt(llr), _fmt(syn),
        f"qkd {q!r}", _fmt(alice), _fmt(bob),
        "syndrome", _fmt(alice)])
    assert out[0] == f"ok code {int(bool(oc.is_regular))}"
    d = out[2].split()
    assert int(d[1]) == p["iterations"] and bool(int(d[2])) == p["syndromes_match"]
    assert [int(x) for x in d[3:]] == oc.decode(llr, syn, p["max_it"], p["thr"], True)["out"].tolist()
    k = out[3].split()
    assert int(k[1]) == p["iterations"] and bool(int(k[3])) == p["keys_match"]
    assert [int(x) for x in out[4].split()[1:]] == syn.tolist()


@pytest.mark.gpu
def test_compat_n10240_decode_trial_batch(driver, golden_code, oracle_code, oracle_mod):
    g = golden_code
    seeds = oracle_mod.seeds(777, 3)
    lines = _code_cmd(10240, 5231, g["chk_off"], g["chk_idx"]) + ["cfg 50 100.0 1 1500 777"]
    want_dec = []
    for s in seeds:
        a, b, q = oracle_mod.keygen(int(s), 10240, 0.08)
        lp = np.log((1 - q) / q)
        llr = np.where(b == 1, -lp, lp)
        syn = oracle_code.syndrome(a)
        lines += ["decode", _fmt(llr), _fmt(syn)]
        want_dec.append(oracle_code.decode(llr, syn, 50, 100.0, True))
    for s in seeds:
        lines.append(f"trial 0.05 {int(s)}")
    lines.append("batch 2 0.02 0.07")
    out = _run(driver, lines)
    dec = [ln for ln in out if ln.startswith("decode")]
    for ln, w in zip(dec, want_dec):
        v = ln.split()
        assert int(v[1]) == w["iters"] and bool(int(v[2])) == w["sp_ok"]
        assert (np.array([int(x) for x in v[3:]]) == w["out"]).all()
    tri = [ln for ln in out if ln.startswith("trial")]
    for ln, s in zip(tri, seeds):
        v = ln.split()
        w = oracle_code.run_trial(0.05, int(s))
        assert (int(v[1]), bool(int(v[2])), bool(int(v[3]))) == (w["iters"], w["sp_ok"], w["key_ok"])
        assert float(v[4]) == w["exact_q"]
    pts = [ln.split() for ln in out if ln.startswith("point")]
    seeds_b = oracle_mod.seeds(777, 1500)
    for k, qn in enumerate([0.02, 0.07]):
        r = oracle_code.trials(qn, seeds_b, k, 50, 100.0, True, threads=min(8, os.cpu_count() or 1))
        st = oracle_mod.batch_stats(r["iters"], r["sp_ok"], r["key_ok"], r["exact_q"], 1500, 50)
        v = pts[k]
        assert int(v[1]) == k
        assert float(v[2]) == st["initial_QBER"]
        assert float(v[3]) == st["iterations_successful_sp_mean"]
        assert float(v[4]) == st["iterations_successful_sp_std_dev"]
        assert int(v[5]) == st["iterations_successful_sp_min"]
        assert int(v[6]) == st["iterations_successful_sp_max"]
        assert float(v[7]) == st["ratio_trials_successful_sp"]
        assert float(v[8]) == st["ratio_trials_successful_ldpc"]


@pytest.mark.gpu
def test_compat_code_cache_survives_address_reuse(driver, oracle_mod):
    """A matrix freed and a different one read at the same address with the same n, m
    (free_matrix_H, array_and_matrix_operations.cpp:88-94; simulation.cpp:108,134) must
    decode on its own adjacency, not on the shim's cached code object."""
    rng = np.random.default_rng(5)
    n, m = 10, 5
    d1 = np.array([[1, 1, 0, 1, 0, 0, 1, 0, 0, 1], [0, 1, 1, 0, 1, 0, 0, 1, 0, 0],
                   [1, 0, 1, 0, 0, 1, 0, 0, 1, 0], [0, 0, 0, 1, 1, 0, 1, 1, 0, 0],
                   [0, 1, 0, 0, 0, 1, 0, 1, 1, 1]], np.uint8)
    d2 = d1[:, rng.permutation(n)]          # same n, m and weights, different adjacency
    assert (d2 != d1).any()
    alice = np.array([1, 0, 1, 1, 0, 0, 1, 1, 0, 1])
    bob = alice.copy()
    bob[3] ^= 1
    q = 0.1
    lp = np.log((1 - q) / q)
    llr = np.where(bob == 1, -lp, lp)
    lines = ["cfg 20 100.0 1 1 777"]
    want = []
    for k, dense in enumerate((d1, d2, d1)):
        off, idx = _dense_lists(dense)
        rows = _code_cmd(n, m, off, idx)
        lines += rows if k == 0 else ["recode"] + rows[1:]
        oc = oracle_mod.Code.from_dense(dense)
        syn = oc.syndrome(alice)
        lines += ["decode", _fmt(llr), _fmt(syn), "syndrome", _fmt(alice)]
        want.append((oc.decode(llr, syn, 20, 100.0, True), syn))
    out = _run(driver, lines)
    dec = [ln.split() for ln in out if ln.startswith("decode")]
    syns = [ln.split()[1:] for ln in out if ln.startswith("syndrome")]
    assert len(dec) == 3 and len(syns) == 3
    for v, s, (w, syn) in zip(dec, syns, want):
        assert int(v[1]) == w["iters"] and bool(int(v[2])) == w["sp_ok"]
        assert [int(x) for x in v[3:]] == w["out"].tolist()
        assert [int(x) for x in s] == syn.tolist()


@pytest.mark.gpu
def test_compat_too_small_qber_throws_reference_message(driver):
    lines = _code_cmd(6, 4, [0, 3, 6, 9, 12], [0, 1, 3, 1, 2, 4, 0, 4, 5, 2, 3, 5])
    p = subprocess.run([driver], input="\n".join(lines + ["cfg 10 100.0 1 1 1", "trial 0.01 5"]) + "\n",
                       text=True, capture_output=True, timeout=120)
    assert "exception Key size '6' is too small for QBER." in p.stdout


@pytest.mark.gpu
def test_compat_variant_selects_minsum(driver, golden_code, oracle_mod):
    """qkd_amd_set_variant("minsum") runs the reference harness on the min-sum
    variant: its batch point equals the library's own min-sum trials; an
    unknown name throws like the reference's errors do. (The shim reads no
    environment variable.)"""
    import qkd_ldpc_amd as Q
    import torch
    g = golden_code
    lines = _code_cmd(10240, 5231, g["chk_off"], g["chk_idx"]) + ["variant minsum", "cfg 50 100.0 1 512 777",
                                                                   "batch 1 0.06"]
    p = subprocess.run([driver], input="\n".join(lines) + "\n", text=True, capture_output=True, timeout=600)
    assert p.returncode == 0, p.stderr
    v = [ln for ln in p.stdout.splitlines() if ln.startswith("point")][0].split()
    H = Q.HMatrix.from_check_lists(10240, g["chk_off"], g["chk_idx"])
    seeds = torch.from_numpy(Q.make_seeds(777, 512).view(np.int64)).cuda()
    r = Q.run_trials(H, seeds, 0.06, 0, 50, variant="minsum")
    torch.cuda.synchronize()
    it = r.iterations.cpu().numpy()
    sp = r.syndromes_match.cpu().numpy().astype(bool)
    st = oracle_mod.batch_stats(it, sp, r.keys_match.cpu().numpy(), r.exact_qber.cpu().numpy(), 512, 50)
    assert float(v[3]) == st["iterations_successful_sp_mean"]
    assert float(v[8]) == st["ratio_trials_successful_ldpc"]
    lines[lines.index("variant minsum")] = "variant bogus"
    p = subprocess.run([driver], input="\n".join(lines) + "\n", text=True, capture_output=True, timeout=600)
    assert "unknown decoder variant 'bogus'" in p.stdout + p.stderr
