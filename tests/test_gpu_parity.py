"""GPU parity: the HIP path (through the C ABI) against the oracle, bit for bit.

Every comparison is exact: decoded bits, iteration counts, syndrome match, key
match, exact QBER and key pairs are integer/byte results of an fp64 algorithm
whose transcendentals are restated bit-exactly (qkd_ldpc_amd/csrc/qkd_math.h).
The oracle is the checker only (oracle/oracle.c, pinned in tests/test_oracle.py).
"""
import os

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


@pytest.fixture(scope="module")
def H(Q, golden_code):
    return Q.HMatrix.from_check_lists(int(golden_code["dims"][0]), golden_code["chk_off"],
                                      golden_code["chk_idx"])


def dev(x, dtype):
    return torch.from_numpy(np.ascontiguousarray(x).astype(dtype)).cuda()


def seeds_dev(seeds):
    return torch.from_numpy(np.ascontiguousarray(seeds, np.uint64).view(np.int64)).cuda()


def llr_of(bob, q):
    lp = np.log((1 - q) / q)
    return np.where(np.asarray(bob) == 1, -lp, lp)


def decode_both(Q, H, ocode, llr, syn, max_it=50, thr=100.0, thr_on=True):
    llr = np.atleast_2d(llr)
    syn = np.atleast_2d(syn)
    r = Q.sum_product_decoding(H, dev(llr, np.float64), dev(syn, np.uint8), max_it, thr, thr_on)
    torch.cuda.synchronize()
    bits = r.bits.cpu().numpy()
    its = r.iterations.cpu().numpy()
    ok = r.syndromes_match.cpu().numpy()
    for f in range(llr.shape[0]):
        want = ocode.decode(llr[f], syn[f], max_it, thr, thr_on)
        assert its[f] == want["iters"], (f, its[f], want["iters"])
        assert bool(ok[f]) == want["sp_ok"], f
        assert (bits[f] == want["out"]).all(), f
    return its, ok


# ---- textbook known answers (BASELINE config 1) ------------------------------------

@pytest.mark.parametrize("case", ["textbook_n6", "textbook_n10"])
def test_textbook_cases(Q, probe, oracle_mod, case):
    p = probe[case]
    dense = np.array(p["dense"], np.uint8)
    H = Q.HMatrix.from_dense_array(dense)
    oc = oracle_mod.Code.from_dense(dense)
    assert H.is_regular == bool(oc.is_regular)
    alice = np.array(p["alice"])
    bob = np.array(p["bob"])
    syn = oc.syndrome(alice)
    its, ok = decode_both(Q, H, oc, llr_of(bob, p["qber"]), syn, p["max_it"], p["thr"], True)
    assert its[0] == p["iterations"] and bool(ok[0]) == p["syndromes_match"]
    r = Q.qkd_ldpc(H, dev(alice[None], np.uint8), dev(bob[None], np.uint8), p["qber"], p["max_it"],
                   p["thr"], True, want_bits=True)
    torch.cuda.synchronize()
    assert int(r.iterations[0]) == p["iterations"]
    assert bool(r.keys_match[0]) == p["keys_match"]
    assert (r.bits.cpu().numpy()[0] == alice).all()


def test_all_dense_matrices_decode(Q, dense_codes, oracle_mod):
    rng = np.random.default_rng(5)
    for name, dense in dense_codes.items():
        H = Q.HMatrix.from_dense_array(dense)
        oc = oracle_mod.Code.from_dense(dense)
        n = dense.shape[1]
        alice = rng.integers(0, 2, (32, n))
        bob = alice ^ (rng.random((32, n)) < 0.15)
        syn = np.stack([oc.syndrome(a) for a in alice])
        decode_both(Q, H, oc, llr_of(bob, 0.15), syn, 20, 100.0, True)


# ---- N=10240 code, LLR entry point ------------------------------------------------

@pytest.mark.parametrize("q_nom,frames", [(0.02, 24), (0.08, 12)])
def test_decode_llr_matches_oracle(Q, H, oracle_code, oracle_mod, q_nom, frames):
    seeds = oracle_mod.seeds(777, frames)
    llr, syn = [], []
    for s in seeds:
        a, b, q = oracle_mod.keygen(int(s), 10240, q_nom)
        llr.append(llr_of(b, q))
        syn.append(oracle_code.syndrome(a))
    decode_both(Q, H, oracle_code, np.stack(llr), np.stack(syn), 50, 100.0, True)


@pytest.mark.parametrize("thr,thr_on,max_it", [(100.0, False, 50), (2.5, True, 50), (100.0, True, 1),
                                               (100.0, True, 3), (0.5, True, 7)])
def test_decode_threshold_and_iteration_caps(Q, H, oracle_code, oracle_mod, thr, thr_on, max_it):
    seeds = oracle_mod.seeds(4242, 6)
    llr, syn = [], []
    for s in seeds:
        a, b, q = oracle_mod.keygen(int(s), 10240, 0.05)
        llr.append(llr_of(b, q))
        syn.append(oracle_code.syndrome(a))
    decode_both(Q, H, oracle_code, np.stack(llr), np.stack(syn), max_it, thr, thr_on)


def test_decode_nan_and_inf_paths(Q, H, oracle_code):
    """Zero LLRs give tanh(0)=0 -> 0/0 = NaN messages; huge LLRs give atanh(+-1) = +-inf.
    The clamp lets NaN through (compare-based) and decisions send NaN to 0."""
    rng = np.random.default_rng(11)
    n, m = 10240, 5231
    llr = rng.normal(2.0, 2.0, (6, n))
    llr[0, rng.integers(0, n, 300)] = 0.0
    llr[1, :] = 0.0
    llr[2, rng.integers(0, n, 500)] = 900.0
    llr[3, rng.integers(0, n, 500)] = -900.0
    llr[4] = np.where(rng.random(n) < 0.5, 1e308, -1e308)
    syn = rng.integers(0, 2, (6, m))
    decode_both(Q, H, oracle_code, llr, syn, 8, 100.0, False)
    decode_both(Q, H, oracle_code, llr, syn, 8, 100.0, True)


def test_syndrome_batch(Q, H, oracle_code):
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 2, (9, 10240))
    got = Q.calculate_syndrome(H, dev(bits, np.uint8)).cpu().numpy()
    for f in range(bits.shape[0]):
        assert (got[f] == oracle_code.syndrome(bits[f])).all()


# ---- key generation (run_trial's keys) -----------------------------------------------

def test_keygen_matches_golden(Q, H, golden_vectors):
    seeds = golden_vectors["kg_seeds"]
    qn = golden_vectors["kg_qnom"]
    k = len(seeds)
    for g in range(len(qn) // k):
        a, b, q = Q.keygen(H, seeds_dev(seeds), float(qn[g * k]))
        torch.cuda.synchronize()
        a = np.packbits(a.cpu().numpy(), axis=1)
        b = np.packbits(b.cpu().numpy(), axis=1)
        assert (a == golden_vectors["kg_alice"][g * k:(g + 1) * k]).all()
        assert (b == golden_vectors["kg_bob"][g * k:(g + 1) * k]).all()
        assert (q.cpu().numpy() == golden_vectors["kg_q"][g * k:(g + 1) * k]).all()


def test_keygen_odd_and_tiny_lengths(Q, oracle_mod):
    """Odd N skips std::shuffle's lone first swap; tiny N exercises ne close to N."""
    rng = np.random.default_rng(9)
    for n, q in [(7, 0.3), (6, 0.5), (9, 1.0), (101, 0.1), (1000, 0.02)]:
        dense = np.zeros((n - 1, n), np.uint8)          # chain code: check j = bits (j, j+1)
        for j in range(n - 1):
            dense[j, j] = dense[j, j + 1] = 1
        H = Q.HMatrix.from_dense_array(dense)
        seeds = rng.integers(0, 2**63, 8, dtype=np.int64).astype(np.uint64)
        a, b, qq = Q.keygen(H, seeds_dev(seeds), q)
        torch.cuda.synchronize()
        for f, s in enumerate(seeds):
            wa, wb, wq = oracle_mod.keygen(int(s), n, q)
            assert (a.cpu().numpy()[f] == wa).all() and (b.cpu().numpy()[f] == wb).all()
            assert qq.cpu().numpy()[f] == wq


def test_qber_too_small_raises(Q, H):
    seeds = seeds_dev(np.arange(4, dtype=np.uint64))
    with pytest.raises(Q.QkdError) as ei:
        Q.run_trials(H, seeds, 1e-5)
    assert "too small" in str(ei.value)


def test_decoded_qber_of_one_rejected(Q, H):
    """Key generation accepts q = 1 (every bit flipped), but a decoded point needs a
    finite log((1 - q) / q): trials and interactive mode reject q >= 1 as
    qkd_qkd_ldpc_batch does, before any key is drawn."""
    seeds = seeds_dev(np.arange(4, dtype=np.uint64))
    with pytest.raises(Q.QkdError) as ei:
        Q.run_trials(H, seeds, 1.0)
    assert ei.value.status == Q._native.ERR_INVALID_ARG
    with pytest.raises(Q.QkdError) as ei:
        Q.interactive_simulation(H, 777, [0.02, 1.0])
    assert ei.value.status == Q._native.ERR_INVALID_ARG


# ---- fused trials: BASELINE configs 2 and 3 per frame ----------------------------------

@pytest.mark.parametrize("sliced", ["1", "0"])
def test_trials_config2_full_batch(Q, H, probe, golden_vectors, monkeypatch, sliced, qkd_opt):
    """sliced 1: the frame syndromes and internal-order keys by
    frame_syn_sliced_kernel (the default); 0: by frame_syn_kernel."""
    qkd_opt("QKD_SYN_SLICED", sliced)
    seeds = Q.make_seeds(777, 4096)
    r = Q.run_trials(H, seeds_dev(seeds), 0.02, 0, 50, 100.0, True)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == golden_vectors["c2_iters"]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == golden_vectors["c2_sp"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c2_ko"]).all()
    q = r.exact_qber.cpu().numpy()
    assert (q == golden_vectors["c2_q"][0]).all()
    st = Q.counters_to_stats(Q.read_counters(r.counters), 4096, 50, float(q[0]))
    p = probe["config2"]
    assert st["sum_iters_sp"] == p["sum_iterations"]
    assert float(f"{st['iterations_successful_sp_mean']:.6g}") == p["mean_6sig"]
    assert float(f"{st['iterations_successful_sp_std_dev']:.6g}") == p["std_6sig"]
    assert st["iterations_successful_sp_min"] == p["min"]
    assert st["iterations_successful_sp_max"] == p["max"]
    assert st["fer"] == p["fer"]


def test_trials_config3_every_point(Q, H, probe, golden_vectors):
    seeds = seeds_dev(Q.make_seeds(777, 10000))
    grid = golden_vectors["c3_qnom"]
    for s, qn in enumerate(grid):
        r = Q.run_trials(H, seeds, float(qn), s, 50, 100.0, True)
        torch.cuda.synchronize()
        assert (r.iterations.cpu().numpy() == golden_vectors["c3_iters"][s]).all(), s
        assert (r.syndromes_match.cpu().numpy().astype(bool) == golden_vectors["c3_sp"][s]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c3_ko"][s]).all()
        st = Q.counters_to_stats(Q.read_counters(r.counters), 10000, 50,
                                 float(r.exact_qber[0]))
        pp = probe["config3"]["points"][s]
        assert abs(st["fer"] - pp["fer"]) < 1e-12
        assert abs(st["iterations_successful_sp_mean"] - pp["mean_it"]) <= 5e-4 + 1e-9


def test_qkd_ldpc_batch_matches_trials(Q, H, golden_vectors):
    """keygen -> qkd_ldpc (byte keys) equals the fused trial path."""
    seeds = seeds_dev(Q.make_seeds(777, 512))
    a, b, q = Q.keygen(H, seeds, 0.02)
    r = Q.qkd_ldpc(H, a, b, float(q[0]), 50, 100.0, True, want_bits=True)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == golden_vectors["c2_iters"][:512]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c2_ko"][:512]).all()
    ok = r.keys_match.cpu().numpy().astype(bool)
    assert (r.bits.cpu().numpy()[ok] == a.cpu().numpy()[ok]).all()


@pytest.mark.parametrize("form", ["bytes", "pack", "bytes_misaligned"])
def test_qkd_ldpc_byte_keys_forms(Q, H, golden_vectors, monkeypatch, form, qkd_opt):
    """qkd_qkd_ldpc_batch's byte keys: packed inside frame_syn_sliced_kernel (the
    default when rows allow 8-byte loads), by pack_kernel first (QKD_SYN_BYTES=0),
    and from 4- but not 8-byte-aligned arrays (pack_kernel, chosen by the launcher);
    1000 frames (the last 16-frame group ragged). Decoded words, iterations and flags
    equal the golden config-2 frames."""
    qkd_opt("QKD_SYN_BYTES", "0" if form == "pack" else "1")
    F = 1000
    seeds = seeds_dev(Q.make_seeds(777, F))
    a, b, q = Q.keygen(H, seeds, 0.02)
    if form == "bytes_misaligned":
        def shift(x):
            buf = torch.empty(x.numel() + 4, dtype=torch.uint8, device=x.device)
            v = buf[4:].view(x.shape)
            v.copy_(x)
            assert v.data_ptr() % 8 == 4
            return v
        a, b = shift(a), shift(b)
    r = Q.qkd_ldpc(H, a, b, float(q[0]), 50, 100.0, True, want_bits=True)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == golden_vectors["c2_iters"][:F]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == golden_vectors["c2_sp"][:F]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c2_ko"][:F]).all()
    ok = r.keys_match.cpu().numpy().astype(bool)
    assert (r.bits.cpu().numpy()[ok] == a.cpu().numpy()[ok]).all()


def test_workspace_and_streams(Q, H, golden_vectors):
    """Two workspaces on two streams give the same per-frame results."""
    seeds = seeds_dev(Q.make_seeds(777, 1024))
    ws1, ws2 = Q.Workspace(H), Q.Workspace(H)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    r1 = Q.run_trials(H, seeds[:512], 0.02, 0, workspace=ws1, stream=s1)
    r2 = Q.run_trials(H, seeds[512:], 0.02, 0, workspace=ws2, stream=s2)
    torch.cuda.synchronize()
    got = np.concatenate([r1.iterations.cpu().numpy(), r2.iterations.cpu().numpy()])
    assert (got == golden_vectors["c2_iters"][:1024]).all()


def test_alist_reader_roundtrip(Q, golden_code, tmp_path):
    from tests.conftest import write_alist
    g = golden_code
    p = os.path.join(tmp_path, "code.alist")
    write_alist(p, 10240, 5231, g["bit_off"], g["bit_idx"], g["chk_off"], g["chk_idx"])
    H = Q.HMatrix.from_alist(p)
    cp, ci, bp, bi = H.adjacency()
    assert (cp == g["chk_off"]).all() and (ci == g["chk_idx"]).all()
    assert (bp == g["bit_off"]).all() and (bi == g["bit_idx"]).all()
    assert not H.is_regular and H.max_bit_nodes_weight == 3 and H.max_check_nodes_weight == 6


# ---- QKD path (keys mode): first-iteration and second-iteration tables -----------------

def _qkd_both(Q, H, oc, alice, bob, q, max_it, thr, thr_on):
    r = Q.qkd_ldpc(H, dev(alice, np.uint8), dev(bob, np.uint8), q, max_it, thr, thr_on,
                   want_bits=True)
    torch.cuda.synchronize()
    its = r.iterations.cpu().numpy()
    sp = r.syndromes_match.cpu().numpy()
    ko = r.keys_match.cpu().numpy()
    bits = r.bits.cpu().numpy()
    for f in range(alice.shape[0]):
        want = oc.qkd_ldpc(alice[f], bob[f], q, max_it, thr, thr_on)
        assert its[f] == want["iters"], (q, thr, thr_on, max_it, f)
        assert bool(sp[f]) == want["sp_ok"] and bool(ko[f]) == want["key_ok"]
        assert (bits[f] == want["out"]).all(), (q, thr, thr_on, max_it, f)


@pytest.mark.parametrize("q", [0.02, 0.08, 0.11, 0.5, 0.7])
@pytest.mark.parametrize("thr,thr_on", [(100.0, True), (2.5, True), (0.7, True), (100.0, False)])
def test_qkd_ldpc_tables_bits_match_oracle(Q, H, oracle_code, oracle_mod, q, thr, thr_on):
    """The QKD path replaces the first check phase by a sign/degree table and the
    second iteration's tanh by a lookup; decoded words, iteration counts and flags
    must still equal the oracle's bit for bit, including failing frames (q >= 0.11),
    log((1-q)/q) = 0 (q = 0.5: NaN messages) and negative LLR magnitudes (q > 0.5)."""
    rng = np.random.default_rng(int(q * 1000) + int(thr * 10) + thr_on)
    f = 3
    alice = rng.integers(0, 2, (f, 10240))
    flips = rng.random((f, 10240)) < min(q, 0.3)
    bob = alice ^ flips
    max_it = 12 if q >= 0.11 else 50
    _qkd_both(Q, H, oracle_code, alice, bob, q, max_it, thr, thr_on)


@pytest.mark.parametrize("max_it", [1, 2, 3])
def test_qkd_ldpc_iteration_caps_inside_tables(Q, H, oracle_code, max_it):
    rng = np.random.default_rng(max_it)
    alice = rng.integers(0, 2, (4, 10240))
    bob = alice ^ (rng.random((4, 10240)) < 0.05)
    _qkd_both(Q, H, oracle_code, alice, bob, 0.05, max_it, 100.0, True)


# ---- the device transcendentals against glibc ---------------------------------------------

def _math_inputs(seed):
    rng = np.random.default_rng(seed)
    u = rng.uniform(-1.0, 1.0, 400_000)
    parts = [u * 60.0, np.ldexp(u, rng.integers(-66, 6, u.size)),
             np.ldexp(np.round(u * 64.0), -5), u, np.ldexp(u, -rng.integers(0, 60, u.size)),
             np.copysign(1.0 - np.ldexp(np.abs(u), -rng.integers(0, 54, u.size)), u),
             np.nextafter(np.copysign(1.0, u), 0.0),
             rng.integers(0, 2**63, u.size, dtype=np.int64).view(np.float64)]
    ex = np.arange(-1075, 1025)
    mant = 1.0 + np.arange(64) / 64.0
    sweep = np.ldexp(mant[None, :], ex[:, None]).ravel()
    sp = np.array([0.0, -0.0, 1.0, -1.0, 22.0, -22.0, 0.5, -0.5, np.inf, -np.inf, np.nan,
                   2.0**-28, 2.0**-55, 2.0**-54, 709.78, -38.0, 0.41422, 5e-324, -5e-324])
    return np.concatenate(parts + [sweep, -sweep, np.nextafter(sweep, 0.0), sp])


@pytest.mark.parametrize("which", ["tanh", "atanh"])
def test_device_math_bit_exact_vs_glibc(Q, oracle_mod, which):
    """The device build of qkd_math.h's flat tanh/atanh (with its shortened
    divisions) equals glibc 2.35 bit for bit (NaN payloads aside)."""
    x = _math_inputs(17 if which == "tanh" else 23)
    dx = torch.from_numpy(x).cuda()
    dy = torch.empty_like(dx)
    Q._native.check(Q._native.lib().qkd_debug_math(0 if which == "tanh" else 1, dx.data_ptr(),
                                                   dy.data_ptr(), x.size, None))
    torch.cuda.synchronize()
    got = dy.cpu().numpy()
    want = oracle_mod.libm(which, x)
    same = (got.view(np.uint64) == want.view(np.uint64)) | (np.isnan(got) & np.isnan(want))
    bad = np.nonzero(~same)[0]
    assert bad.size == 0, [(float.hex(x[i]), float.hex(got[i]), float.hex(want[i])) for i in bad[:5]]


@pytest.mark.parametrize("mode", ["fast", "lanes", "matrix", "replay", "serial"])
def test_keygen_kernels_agree_with_oracle(Q, oracle_mod, monkeypatch, mode, qkd_opt):
    """The two-wave jump-ahead generator (default), its serial regeneration
    (taken after a Lemire rejection; forced here), the one-wave generator with
    polynomial and matrix jumps, and the one-thread-per-frame kernel all
    reproduce run_trial's keys."""
    if mode != "fast":
        qkd_opt("QKD_KEYGEN", mode)
    rng = np.random.default_rng(31)
    for n, q in [(2, 0.5), (3, 1.0), (6, 0.5), (10, 1.0), (64, 0.1), (65, 0.5), (127, 0.3),
                 (1001, 0.02), (4100, 1.0), (10240, 0.3), (10240, 0.45)]:
        dense = np.zeros((n - 1, n), np.uint8)
        for j in range(n - 1):
            dense[j, j] = dense[j, j + 1] = 1
        H = Q.HMatrix.from_dense_array(dense)
        seeds = rng.integers(0, 2**63, 6, dtype=np.int64).astype(np.uint64)
        a, b, qq = Q.keygen(H, seeds_dev(seeds), q)
        torch.cuda.synchronize()
        a, b, qq = a.cpu().numpy(), b.cpu().numpy(), qq.cpu().numpy()
        for f, s in enumerate(seeds):
            wa, wb, wq = oracle_mod.keygen(int(s), n, q)
            assert (a[f] == wa).all() and (b[f] == wb).all(), (mode, n, q, f)
            assert qq[f] == wq


def test_irregular_high_degree_bits_keys_path(Q, oracle_mod, tmp_path):
    """Bit degrees 2..6 (beyond the unrolled rows and the table limit): the fused
    trial path takes the general first/second iterations and the bit phase's
    tail rows; results equal the oracle."""
    from conftest import write_alist
    rng = np.random.default_rng(21)
    n, m = 3000, 1500
    degs = rng.choice([2, 3, 4, 5, 6], size=n, p=[0.2, 0.4, 0.2, 0.1, 0.1])
    rows = [[] for _ in range(m)]
    for i in range(n):
        for j in rng.choice(m, size=degs[i], replace=False):
            rows[j].append(i)
    rows = [sorted(r) for r in rows if r] 
    m = len(rows)
    co = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
    ci = np.concatenate(rows).astype(np.int32)
    H = Q.HMatrix.from_check_lists(n, co, ci)
    cptr, cidx, bptr, bidx = H.adjacency()
    p = str(tmp_path / "irr.alist")
    write_alist(p, n, m, bptr, bidx, cptr, cidx, pad=False)
    oc = oracle_mod.Code.from_alist(p)
    seeds = oracle_mod.seeds(31, 24)
    for q in (0.02, 0.06):
        r = Q.run_trials(H, seeds_dev(seeds), q, 0, 30)
        torch.cuda.synchronize()
        want = oc.trials(q, seeds, 0, 30, 100.0, True)
        assert (r.iterations.cpu().numpy() == want["iters"]).all()
        assert (r.syndromes_match.cpu().numpy().astype(bool) == want["sp_ok"]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == want["key_ok"]).all()


def test_qkd_ldpc_unaligned_key_bytes(Q, H, golden_vectors):
    """Key bytes whose rows start off a 16-byte boundary take the packing kernel's
    byte path (the wide path needs N % 32 == 0 and aligned arrays); same outputs."""
    seeds = seeds_dev(Q.make_seeds(777, 64))
    a, b, q = Q.keygen(H, seeds, 0.02)
    buf_a = torch.zeros(64 * 10240 + 16, dtype=torch.uint8, device="cuda")
    buf_b = torch.zeros(64 * 10240 + 16, dtype=torch.uint8, device="cuda")
    ua = buf_a[3:3 + 64 * 10240].view(64, 10240)
    ub = buf_b[5:5 + 64 * 10240].view(64, 10240)
    ua.copy_(a)
    ub.copy_(b)
    r = Q.qkd_ldpc(H, ua, ub, float(q[0]), 50, 100.0, True, want_bits=True)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == golden_vectors["c2_iters"][:64]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c2_ko"][:64]).all()
    assert (r.bits.cpu().numpy() == a.cpu().numpy()).all()


def _chain_code(Q, n):
    """H of the chain code (check j = bits j, j + 1), from check lists (a dense
    array of N ~ 70,000 would take gigabytes)."""
    co = (2 * np.arange(n, dtype=np.int32))
    ci = np.stack([np.arange(n - 1), np.arange(1, n)], 1).reshape(-1).astype(np.int32)
    return Q.HMatrix.from_check_lists(n, co, ci)


@pytest.mark.parametrize("mode", ["fast", "replay"])
def test_keygen_beyond_65536_bits(Q, oracle_mod, monkeypatch, mode, qkd_opt):
    """The two-wave generator at and past N = 65536, where its Lemire products leave
    32 bits (keygen_split_kernel<false>: binary64 quotients, 64-bit draw indices),
    and its serial regeneration path there: keys and exact QBER equal run_trial's."""
    if mode != "fast":
        qkd_opt("QKD_KEYGEN", mode)
    rng = np.random.default_rng(65)
    for n, q in [(65536, 0.02), (65536, 0.05), (65537, 0.02), (70001, 0.03)]:
        H = _chain_code(Q, n)
        seeds = rng.integers(0, 2**63, 3, dtype=np.int64).astype(np.uint64)
        a, b, qq = Q.keygen(H, seeds_dev(seeds), q)
        torch.cuda.synchronize()
        a, b, qq = a.cpu().numpy(), b.cpu().numpy(), qq.cpu().numpy()
        for f, s in enumerate(seeds):
            wa, wb, wq = oracle_mod.keygen(int(s), n, q)
            assert (a[f] == wa).all() and (b[f] == wb).all(), (mode, n, q, f)
            assert qq[f] == wq


def test_trials_beyond_65536_bits(Q, oracle_mod, tmp_path):
    """run_trials on a 70,001-bit code (past the split decoder's N limit: the classic
    kernel, with the binary64-quotient key generator): per-frame iterations and flags
    equal the oracle's."""
    from conftest import write_alist
    n = 70001
    H = _chain_code(Q, n)
    cptr, cidx, bptr, bidx = H.adjacency()
    p = str(tmp_path / "chain.alist")
    write_alist(p, n, n - 1, bptr, bidx, cptr, cidx, pad=False)
    oc = oracle_mod.Code.from_alist(p)
    seeds = oracle_mod.seeds(70, 4)
    for q, max_it in [(0.001, 6), (0.02, 4)]:
        r = Q.run_trials(H, seeds_dev(seeds), q, 0, max_it, 100.0, True)
        torch.cuda.synchronize()
        want = oc.trials(q, seeds, 0, max_it, 100.0, True, threads=4)
        assert (r.iterations.cpu().numpy() == want["iters"]).all(), q
        assert (r.syndromes_match.cpu().numpy().astype(bool) == want["sp_ok"]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == want["key_ok"]).all()


def test_decoder_timing_counts_launches(Q, golden_code):
    """qkd_debug_decoder_timing (the bench's live kernel time): pairs of HIP events
    around each decoder launch; 600 calls cross the pool's fold point (256 pairs) and
    every launch is counted once, with a positive total."""
    import ctypes as C
    g = golden_code
    H = Q.HMatrix.from_check_lists(int(g["dims"][0]), g["chk_off"], g["chk_idx"])
    ws = Q.Workspace(H)
    seeds = seeds_dev(Q.make_seeds(777, 64))
    alice, bob, q = Q.keygen(H, seeds, 0.02, 0, workspace=ws)
    L = Q._native.lib()
    tot, n = C.c_double(0), C.c_uint64(0)
    Q._native.check(L.qkd_debug_decoder_timing(ws.handle, 1, C.byref(tot), C.byref(n)))
    for k in range(600):
        Q.qkd_ldpc(H, alice, bob, float(q[0].item()), workspace=ws)
    Q._native.check(L.qkd_debug_decoder_timing(ws.handle, 0, C.byref(tot), C.byref(n)))
    assert n.value == 600 and tot.value > 0
    # off again: no events recorded, nothing counted
    Q.qkd_ldpc(H, alice, bob, float(q[0].item()), workspace=ws)
    Q._native.check(L.qkd_debug_decoder_timing(ws.handle, 0, C.byref(tot), C.byref(n)))
    assert n.value == 0 and tot.value == 0.0
    ws.close()
