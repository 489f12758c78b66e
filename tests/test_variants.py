"""Decoder variants (include/qkd_ldpc.h QKD_VARIANT_*).

The reference has one decoder, binary64 sum-product; that is QKD_VARIANT_SP_F64
and the parity suites (test_gpu_parity.py) hold it to the reference bit for bit.
The variants are build-defined:
  * min-sum: checked bit for bit against its numpy binary32 specification
    (oracle/variants.py) - decoded words, iteration counts, flags;
  * binary32 sum-product: checked bit for bit against its numpy specification
    with the device's own elementwise tanhf/atanhf plugged in (OCML has no
    bit-exact CPU twin here; those two functions are checked separately against
    numpy's float32 ones to ~1 ulp), and against the reference decoder's outcome
    where the code has margin.
Frame error rates of both against the reference curve are reported by bench.py.
"""
import numpy as np
import pytest

from oracle.variants import MinSumModel


@pytest.fixture(scope="module")
def ms_model(golden_code):
    return MinSumModel(int(golden_code["dims"][0]), int(golden_code["dims"][1]),
                       golden_code["chk_off"], golden_code["chk_idx"])


def _frames(oracle_mod, q, count, seed=777):
    A, B = [], []
    for s in oracle_mod.seeds(seed, count):
        a, b, qq = oracle_mod.keygen(int(s), 10240, q)
        A.append(a)
        B.append(b)
    return np.array(A, np.uint8), np.array(B, np.uint8), qq


# ---- CPU: the specification itself ------------------------------------------------

def test_minsum_model_decodes_low_qber(ms_model, oracle_mod):
    A, B, q = _frames(oracle_mod, 0.03, 8)
    lp = np.log((1 - q) / q)
    llr = np.where(B == 1, -lp, lp)
    bits, it, ok = ms_model.decode(llr, ms_model.syndrome(A))
    assert ok.all() and (bits == A).all()
    assert (it >= 2).all() and (it <= 10).all()


def test_minsum_model_syndrome_matches_oracle(ms_model, oracle_code):
    rng = np.random.default_rng(5)
    bits = rng.integers(0, 2, (3, 10240)).astype(np.uint8)
    got = ms_model.syndrome(bits)
    for f in range(3):
        assert (got[f] == oracle_code.syndrome(bits[f])).all()


def test_decoder_flags_validation():
    import qkd_ldpc_amd as Q
    assert Q.decoder_flags(True, "minsum", minsum_self_correct=True) == 0x1 | 0x20 | (1 << 24)
    with pytest.raises(ValueError):
        Q.decoder_flags(True, "sp_f32", minsum_self_correct=True)
    assert Q.decoder_flags(True, "sp_f64") == 0x1
    assert Q.decoder_flags(False, "minsum") == 0x20
    assert Q.decoder_flags(True, "minsum", 0.5) == 0x1 | 0x20 | (128 << 8)
    with pytest.raises(ValueError):
        Q.decoder_flags(True, "bogus")
    with pytest.raises(ValueError):
        Q.decoder_flags(True, "sp_f32", 0.5)
    with pytest.raises(ValueError):
        Q.decoder_flags(True, "minsum", 0.3)     # not k/256


# ---- GPU ---------------------------------------------------------------------------

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


def _dev(x, dtype):
    return torch.from_numpy(np.ascontiguousarray(x).astype(dtype)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("q,max_it,thr,thr_on,scale,offset", [
    (0.02, 50, 100.0, True, None, None),
    (0.06, 50, 100.0, True, None, None),
    (0.08, 50, 100.0, True, 0.8125, None),
    (0.08, 7, 2.5, True, 0.5, None),
    (0.05, 50, 0.0, False, None, None),
    (0.10, 3, 0.7, True, 255 / 256, None),
    (0.08, 50, 100.0, True, 0.9375, 0.25),
    (0.07, 50, 2.5, True, 1.0 - 1 / 256, 3.0),
])
@pytest.mark.parametrize("store", ["split", "lds", "global"])
def test_minsum_llr_bit_exact(Q, H, ms_model, oracle_mod, monkeypatch, store, q, max_it, thr, thr_on,
                              scale, offset, qkd_opt):
    """The three min-sum kernels: the split skeleton (one binary32 slot per
    edge, all in LDS; the default where it fits), the frame state in LDS
    (per-check min1/min2/argmin/signs) and the per-edge global message store;
    plain normalised and offset min-sum."""
    if store != "split":
        qkd_opt("QKD_MINSUM_STORE", store)
    A, B, qq = _frames(oracle_mod, q, 48, seed=int(q * 1000) + max_it)
    lp = np.log((1 - qq) / qq)
    llr = np.where(B == 1, -lp, lp)
    syn = ms_model.syndrome(A)
    r = Q.sum_product_decoding(H, _dev(llr, np.float64), _dev(syn, np.uint8), max_it,
                               thr if thr_on else 100.0, thr_on, variant="minsum",
                               minsum_scale=scale, minsum_offset=offset)
    torch.cuda.synchronize()
    want_bits, want_it, want_ok = ms_model.decode(llr, syn, max_it, thr, thr_on,
                                                  0.8125 if scale is None else scale, offset or 0.0)
    assert (r.iterations.cpu().numpy() == want_it).all()
    assert (r.syndromes_match.cpu().numpy() == want_ok).all()
    assert (r.bits.cpu().numpy() == want_bits).all()


@pytest.mark.gpu
@pytest.mark.parametrize("q,max_it,thr,thr_on,scale", [
    (0.05, 50, 100.0, True, None), (0.08, 50, 100.0, True, 0.875), (0.08, 50, 100.0, True, 0.75),
    (0.07, 6, 2.5, True, 1.0 - 1 / 256), (0.06, 50, 0.0, False, None)])
@pytest.mark.parametrize("store", ["split", "lds"])
def test_minsum_self_corrected_bit_exact(Q, H, ms_model, oracle_mod, monkeypatch, store, q, max_it, thr, thr_on,
                                         scale, qkd_opt):
    """Self-corrected min-sum (QKD_MINSUM_SELF_CORRECT; the split kernel's per-task
    ballot words or the LDS-state kernel) against its specification: erasures of
    sign-flipped b2c from the second iteration on."""
    if store != "split":
        qkd_opt("QKD_MINSUM_STORE", store)
    A, B, qq = _frames(oracle_mod, q, 48, seed=int(q * 1000) + 31 + max_it)
    lp = np.log((1 - qq) / qq)
    llr = np.where(B == 1, -lp, lp)
    syn = ms_model.syndrome(A)
    r = Q.sum_product_decoding(H, _dev(llr, np.float64), _dev(syn, np.uint8), max_it,
                               thr if thr_on else 100.0, thr_on, variant="minsum",
                               minsum_scale=scale, minsum_self_correct=True)
    torch.cuda.synchronize()
    want_bits, want_it, want_ok = ms_model.decode(llr, syn, max_it, thr, thr_on,
                                                  0.8125 if scale is None else scale, 0.0, self_correct=True)
    assert (r.iterations.cpu().numpy() == want_it).all()
    assert (r.syndromes_match.cpu().numpy() == want_ok).all()
    assert (r.bits.cpu().numpy() == want_bits).all()
    # and the keys path
    r = Q.qkd_ldpc(H, _dev(A, np.uint8), _dev(B, np.uint8), float(qq), max_it,
                   thr if thr_on else 100.0, thr_on, want_bits=True, variant="minsum",
                   minsum_scale=scale, minsum_self_correct=True)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == want_it).all()
    assert (r.bits.cpu().numpy() == want_bits).all()


@pytest.mark.gpu
def test_minsum_self_corrected_needs_lds_state(Q, H, monkeypatch, qkd_opt):
    """The global-store min-sum has no self-correction: the call fails loudly."""
    qkd_opt("QKD_MINSUM_STORE", "global")
    llr = torch.ones((2, 10240), dtype=torch.float64, device="cuda")
    syn = torch.zeros((2, 5231), dtype=torch.uint8, device="cuda")
    with pytest.raises(Q.QkdError):
        Q.sum_product_decoding(H, llr, syn, 5, 100.0, True, variant="minsum", minsum_self_correct=True)


@pytest.mark.gpu
@pytest.mark.parametrize("store,q,offset", [("split", 0.07, None), ("split", 0.02, None), ("split", 0.08, 0.25),
                                            ("lds", 0.07, None)])
def test_minsum_keys_path_bit_exact(Q, H, ms_model, oracle_mod, monkeypatch, store, q, offset, qkd_opt):
    """qkd_ldpc (packed-key path, LLR = +-float(log_p); the split kernel folds
    its first iteration) equals the specification."""
    if store != "split":
        qkd_opt("QKD_MINSUM_STORE", store)
    A, B, qq = _frames(oracle_mod, q, 48, seed=4242 + int(q * 100))
    r = Q.qkd_ldpc(H, _dev(A, np.uint8), _dev(B, np.uint8), float(qq), 50, 100.0, True,
                   want_bits=True, variant="minsum", minsum_offset=offset)
    torch.cuda.synchronize()
    lp = np.log((1 - qq) / qq)
    llr = np.where(B == 1, -lp, lp)
    want_bits, want_it, want_ok = ms_model.decode(llr, ms_model.syndrome(A), scale=0.8125, offset=offset or 0.0)
    assert (r.iterations.cpu().numpy() == want_it).all()
    assert (r.syndromes_match.cpu().numpy() == want_ok).all()
    assert (r.bits.cpu().numpy() == want_bits).all()
    assert (r.keys_match.cpu().numpy() == (want_bits == A).all(axis=1)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("store", ["split", "lds", "global"])
def test_minsum_small_codes_bit_exact(Q, dense_codes, monkeypatch, store, qkd_opt):
    if store != "split":
        qkd_opt("QKD_MINSUM_STORE", store)
    rng = np.random.default_rng(17)
    for name, dense in dense_codes.items():
        m, n = dense.shape
        co = np.concatenate([[0], np.cumsum(dense.sum(axis=1))]).astype(np.int32)
        ci = np.concatenate([np.nonzero(r)[0] for r in dense]).astype(np.int32)
        model = MinSumModel(n, m, co, ci)
        Hs = Q.HMatrix.from_dense_array(dense)
        llr = rng.normal(0.8, 1.5, (16, n))
        syn = rng.integers(0, 2, (16, m)).astype(np.uint8)
        r = Q.sum_product_decoding(Hs, _dev(llr, np.float64), _dev(syn, np.uint8), 20, 3.0, True,
                                   variant="minsum")
        torch.cuda.synchronize()
        wb, wi, wo = model.decode(llr, syn, 20, 3.0, True, 0.8125)
        assert (r.iterations.cpu().numpy() == wi).all(), name
        assert (r.syndromes_match.cpu().numpy() == wo).all(), name
        assert (r.bits.cpu().numpy() == wb).all(), name


def _dev_math(which):
    from qkd_ldpc_amd import _native as N

    def f(v):
        x = torch.from_numpy(np.ascontiguousarray(v, np.float64).ravel()).cuda()
        y = torch.empty_like(x)
        N.check(N.lib().qkd_debug_math(which, x.data_ptr(), y.data_ptr(), x.numel(), None))
        torch.cuda.synchronize()
        return y.cpu().numpy().astype(np.float32).reshape(np.shape(v))
    return f


@pytest.mark.gpu
def test_sp_f32_elementwise_math_close_to_numpy(Q):
    """The binary32 variant's two steps (Gallager form) against binary64 numpy: the
    published sign(x) psi(|x|) and phi(S ln 2)."""
    from oracle.variants import _phi_out_np, _psi_np
    # binary32 arguments (the device rounds its inputs to binary32; phi(x) ~ 2 e^-x
    # turns an argument rounding into a relative error of x 2^-24)
    x = np.concatenate([np.linspace(-100, 100, 20001), np.geomspace(1e-12, 1, 20001),
                        -np.geomspace(1e-12, 1, 2001), [0.0, -0.0, 1.0, -1.0, 80.0, 1e-30]])
    s = np.concatenate([np.geomspace(1e-30, 200, 40001), [0.0]])
    x = x.astype(np.float32).astype(np.float64)
    s = s.astype(np.float32).astype(np.float64)
    with np.errstate(all="ignore"):
        pub = _dev_math(2)(x)
        out = _dev_math(3)(s)
    want_pub, want_out = _psi_np(x), _phi_out_np(s)
    assert (np.sign(pub[x != 0]) == np.sign(x[x != 0])).all()
    # the variant's phi is held to 5e-6 relative (qkd_decode.h, RuleMath<kRuleSp32>:
    # no argument split in 2^-(x log2 e), short series)
    assert np.allclose(pub, want_pub, rtol=5e-6, atol=0)
    fin = np.isfinite(want_out)
    assert np.allclose(out[fin], want_out[fin], rtol=5e-6, atol=1e-37)
    assert np.isinf(out[~fin]).all()


@pytest.mark.gpu
def test_sp_f32_pair_equals_scalar_forms(Q):
    """The check phase's packed evaluation of one input psi and one output phi
    (RuleMath<kRuleSp32>::pair) equals the scalar forms the specification calls
    (debug math 2 / 3) bit for bit, branch edges and clamps included."""
    rng = np.random.default_rng(23)
    n = 1 << 19
    x = np.exp(rng.uniform(np.log(1e-35), np.log(150.0), n)) * rng.choice([-1.0, 1.0], n)
    s = np.exp(rng.uniform(np.log(1e-35), np.log(300.0), n))
    sx = np.array([0.0, -0.0, 1e-30, 1e-31, 0.03125, np.nextafter(0.03125, 0), 2.0, np.nextafter(2.0, 0),
                   80.0, 81.0, -80.0, 1e-45])
    ss = np.array([0.0, 1e-40, 0.03125 / np.log(2), 2.0 / np.log(2), 2.8853900817779268, 115.0, 116.0,
                   np.inf, 1e-30, 1.0, 1e-45, 300.0])
    x[: sx.size] = sx
    s[: ss.size] = ss
    xs = np.empty(2 * n)
    xs[0::2], xs[1::2] = x, s
    dx = torch.from_numpy(xs).cuda()
    out = {}
    for which in (12, 13):
        dy = torch.empty_like(dx)
        Q._native.check(Q._native.lib().qkd_debug_math(which, dx.data_ptr(), dy.data_ptr(), dx.numel(), None))
        torch.cuda.synchronize()
        out[which] = dy.cpu().numpy().view(np.uint64)
    bad = np.nonzero(out[12] != out[13])[0]
    assert bad.size == 0, (bad[:8], xs[bad[:8]])


@pytest.mark.gpu
@pytest.mark.parametrize("q,max_it,thr,thr_on", [(0.05, 50, 100.0, True), (0.08, 50, 100.0, True),
                                                 (0.07, 9, 3.0, True), (0.06, 50, 0.0, False)])
def test_sp_f32_bit_exact_with_device_math(Q, H, ms_model, oracle_mod, q, max_it, thr, thr_on):
    from oracle.variants import sp_f32_decode
    A, B, qq = _frames(oracle_mod, q, 24, seed=int(q * 1000) + 7)
    lp = np.log((1 - qq) / qq)
    llr = np.where(B == 1, -lp, lp)
    syn = ms_model.syndrome(A)
    r = Q.sum_product_decoding(H, _dev(llr, np.float64), _dev(syn, np.uint8), max_it,
                               thr if thr_on else 100.0, thr_on, variant="sp_f32")
    torch.cuda.synchronize()
    wb, wi, wo = sp_f32_decode(ms_model, llr, syn, max_it, thr, thr_on,
                               tanh_half=_dev_math(2), two_atanh=_dev_math(3))
    assert (r.iterations.cpu().numpy() == wi).all()
    assert (r.syndromes_match.cpu().numpy() == wo).all()
    assert (r.bits.cpu().numpy() == wb).all()


@pytest.mark.gpu
@pytest.mark.parametrize("q,max_it,thr", [(0.03, 50, 100.0), (0.08, 50, 100.0), (0.06, 2, 3.0), (0.07, 1, 100.0)])
def test_sp_f32_keys_path_bit_exact(Q, H, ms_model, oracle_mod, q, max_it, thr):
    """qkd_ldpc with the binary32 rule: its first check phase is folded into the first
    bit phase (messages +-C_d from a per-degree table the kernel evaluates with the same
    device steps), so the keys path must equal the unfolded specification bit for bit."""
    from oracle.variants import sp_f32_decode
    A, B, qq = _frames(oracle_mod, q, 24, seed=int(q * 1000) + max_it)
    r = Q.qkd_ldpc(H, _dev(A, np.uint8), _dev(B, np.uint8), float(qq), max_it, thr, True,
                   want_bits=True, variant="sp_f32")
    torch.cuda.synchronize()
    lp = np.log((1 - qq) / qq)
    llr = np.where(B == 1, -lp, lp)
    wb, wi, wo = sp_f32_decode(ms_model, llr, ms_model.syndrome(A), max_it, thr, True,
                               tanh_half=_dev_math(2), two_atanh=_dev_math(3))
    assert (r.iterations.cpu().numpy() == wi).all()
    assert (r.syndromes_match.cpu().numpy() == wo).all()
    assert (r.bits.cpu().numpy() == wb).all()
    assert (r.keys_match.cpu().numpy() == (wb == A).all(axis=1)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("q", [0.02, 0.05])
def test_sp_f32_tracks_reference(Q, H, q):
    """binary32 sum-product (Gallager form): where the code has margin it decodes every
    frame, and to the same iteration count as the reference decoder on nearly all."""
    seeds = torch.from_numpy(Q.make_seeds(777, 1024).view(np.int64)).cuda()
    ref = Q.run_trials(H, seeds, q)
    f32 = Q.run_trials(H, seeds, q, variant="sp_f32")
    torch.cuda.synchronize()
    assert f32.syndromes_match.cpu().numpy().all() and f32.keys_match.cpu().numpy().all()
    same = (ref.iterations.cpu().numpy() == f32.iterations.cpu().numpy()).mean()
    assert same >= 0.97, same


@pytest.mark.gpu
def test_variant_trials_counters(Q, H):
    """The fused trial path with a variant: counters agree with the per-frame outputs."""
    seeds = torch.from_numpy(Q.make_seeds(777, 512).view(np.int64)).cuda()
    r = Q.run_trials(H, seeds, 0.06, variant="minsum")
    torch.cuda.synchronize()
    c = Q.read_counters(r.counters)
    it = r.iterations.cpu().numpy().astype(np.int64)
    sp = r.syndromes_match.cpu().numpy().astype(bool)
    ko = r.keys_match.cpu().numpy().astype(bool)
    assert c.frames == 512 and c.sp_ok == sp.sum() and c.ldpc_ok == (sp & ko).sum()
    assert c.sum_iters == it[sp].sum()


# ---- high-rate codes: check degrees in the 16 and 64 buckets -------------------------------

def _high_rate_code(n, dc, seed):
    """(3, dc)-regular code: each bit (random order) joins the three distinct checks
    with the most free places (random tie-break), so no edge repeats and every
    check ends with exactly dc bits. -> (m, check_ptr, check_idx), rows ascending."""
    rng = np.random.default_rng(seed)
    m = n * 3 // dc
    assert m * dc == n * 3
    free = np.full(m, dc)
    rows = [[] for _ in range(m)]
    for i in rng.permutation(n):
        key = free + rng.random(m) * 0.5
        for j in np.argsort(-key)[:3]:
            rows[j].append(int(i))
            free[j] -= 1
    assert (free == 0).all()
    ci = np.concatenate([sorted(r) for r in rows]).astype(np.int32)
    return m, np.arange(0, m * dc + 1, dc, dtype=np.int32), ci


@pytest.mark.gpu
@pytest.mark.parametrize("n,dc,q", [(2048, 64, 0.002), (2048, 32, 0.005), (1536, 12, 0.02)])
@pytest.mark.parametrize("path", ["llr", "keys"])
def test_sp_f32_high_check_degree_bit_exact(Q, oracle_mod, n, dc, q, path):
    """sp_f32 on codes whose check degree lands in the 16- and 64-entry buckets of the
    check phase (R = 0.95 at degree 64, the reference config's code_rate 0.95 row):
    the extrinsic-sum weights of those buckets come from a 64-bit segment mask
    (decode_split.hip SegWeights); bit for bit against the specification."""
    from oracle.variants import sp_f32_decode
    m, cp, ci = _high_rate_code(n, dc, seed=dc)
    model = MinSumModel(n, m, cp, ci)
    Hh = Q.HMatrix.from_check_lists(n, cp, ci)
    assert Hh.max_check_nodes_weight == dc
    A, B = [], []
    for s in oracle_mod.seeds(dc + 5, 16):
        a, b, qq = oracle_mod.keygen(int(s), n, q)
        A.append(a)
        B.append(b)
    A, B = np.array(A, np.uint8), np.array(B, np.uint8)
    lp = np.log((1 - qq) / qq)
    llr = np.where(B == 1, -lp, lp)
    syn = model.syndrome(A)
    if path == "llr":
        r = Q.sum_product_decoding(Hh, _dev(llr, np.float64), _dev(syn, np.uint8), 30, 100.0, True,
                                   variant="sp_f32")
    else:
        r = Q.qkd_ldpc(Hh, _dev(A, np.uint8), _dev(B, np.uint8), float(qq), 30, 100.0, True,
                       want_bits=True, variant="sp_f32")
    torch.cuda.synchronize()
    wb, wi, wo = sp_f32_decode(model, llr, syn, 30, 100.0, True,
                               tanh_half=_dev_math(2), two_atanh=_dev_math(3))
    assert (r.iterations.cpu().numpy() == wi).all()
    assert (r.syndromes_match.cpu().numpy() == wo).all()
    assert (r.bits.cpu().numpy() == wb).all()
    assert wo.mean() > 0.5       # the frames mostly decode: the check phase's sums matter


@pytest.mark.gpu
@pytest.mark.parametrize("n,dc,q", [(2048, 64, 0.002), (1536, 12, 0.02)])
def test_sp_f64_high_check_degree_matches_oracle(Q, oracle_mod, tmp_path, n, dc, q):
    """The reference decoder on the same high-rate codes: fused trials equal the oracle."""
    from conftest import write_alist
    m, cp, ci = _high_rate_code(n, dc, seed=dc)
    Hh = Q.HMatrix.from_check_lists(n, cp, ci)
    cptr, cidx, bptr, bidx = Hh.adjacency()
    p = str(tmp_path / "hr.alist")
    write_alist(p, n, m, bptr, bidx, cptr, cidx)
    oc = oracle_mod.Code.from_alist(p)
    seeds = oracle_mod.seeds(41, 24)
    r = Q.run_trials(Hh, torch.from_numpy(seeds.view(np.int64)).cuda(), q, 0, 30)
    torch.cuda.synchronize()
    want = oc.trials(q, seeds, 0, 30, 100.0, True)
    assert (r.iterations.cpu().numpy() == want["iters"]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == want["sp_ok"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == want["key_ok"]).all()
