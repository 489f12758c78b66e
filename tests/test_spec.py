"""Speculative interval iterations (qkd_ldpc_amd/csrc/qkd_spec.h, decode_split.hip).

The QKD path first decodes each frame with binary32 intervals that must contain
the reference's binary64 messages; a frame whose hard decisions the intervals
cannot certify is decoded again exactly. Outputs must be bit-exact either way:
every comparison below is exact (iteration counts, flags, decoded bits), against
the golden vectors of the pinned oracle or the oracle itself, at several caps
(QKD_SPEC_CAP; 0 = exact iterations only).
"""
import ctypes as C

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


def seeds_dev(seeds):
    return torch.from_numpy(np.ascontiguousarray(seeds, np.uint64).view(np.int64)).cuda()


def phi64(x):
    """phi(x) = -ln tanh(x/2) = log1p(2u / (1 - u)), u = e^-x, in binary64."""
    x = np.asarray(x, np.float64)
    u = np.exp(-x)
    return np.log1p(2.0 * u / -np.expm1(-x))


def replays(Q, ws, reset=True):
    v = C.c_uint64(0)
    Q._native.check(Q._native.lib().qkd_debug_spec_replays(ws.handle, C.byref(v), int(reset)))
    return v.value


LN2 = np.log(2.0)


def psi_units(x, direction):
    """Natural-unit sums as the log2-domain binary32 the output form takes
    (x / ln 2), rounded down (-1), to nearest (0) or up (+1)."""
    f = (np.asarray(x, np.float64) / LN2).astype(np.float32)
    if direction:
        f = np.nextafter(f, np.float32(np.inf if direction > 0 else 0.0))
    return f.astype(np.float64)


def device_phi(Q, which, a, b):
    x = np.empty(2 * a.size, np.float64)
    x[0::2] = a
    x[1::2] = b
    dx = torch.from_numpy(x).cuda()
    dy = torch.empty_like(dx)
    Q._native.check(Q._native.lib().qkd_debug_math(which, dx.data_ptr(), dy.data_ptr(), dx.numel(), None))
    torch.cuda.synchronize()
    y = dy.cpu().numpy()
    return y[0::2], y[1::2]


@pytest.mark.parametrize("rel", [0.0, 1e-7, 1e-5, 1e-3, 0.5])
def test_phi_bounds_contain_phi(Q, rel):
    """phi_bounds (input side) and phi_bounds_out (output side) bracket phi over
    [a, b] for a dense sweep of a (binary32) in [1e-30, 120]; the value checked is
    phi at both ends (phi is monotone, so the ends are its extremes)."""
    rng = np.random.default_rng(7)
    a = np.concatenate([
        np.exp(rng.uniform(np.log(1e-30), np.log(120.0), 1000000)),
        rng.uniform(0.0, 5.0, 1000000),
        np.array([0.35, 2.0, 4.0, 80.0, 1.0, 0.5], np.float64),
    ]).astype(np.float32).astype(np.float64)
    b = (a * (1.0 + rel)).astype(np.float32).astype(np.float64)
    b = np.maximum(a, b)
    for which in (4, 5):
        # the output form works on log2-domain sums: an enclosing interval of
        # [a, b] for containment, the nearest value (its exact phi) for headroom
        if which == 4:
            lo, hi = device_phi(Q, which, a, b)
        else:
            lo, hi = device_phi(Q, which, psi_units(a, -1), psi_units(b, 1))
        pa, pb = phi64(a), phi64(b)
        assert (lo <= pb).all(), (which, a[lo > pb][:5], lo[lo > pb][:5], pb[lo > pb][:5])
        assert (hi >= pa).all(), (which, a[hi < pa][:5], hi[hi < pa][:5], pa[hi < pa][:5])
        assert (lo >= 0).all()
        if rel == 0.0:
            if which == 5:
                an = psi_units(a, 0)
                lo, hi = device_phi(Q, which, an, an)
                pa = phi64(an * LN2)
            fin0 = (a < 70) & (pa > 1e-30)
            # headroom: how much of the 2^-20 allowance the evaluation uses
            # (hi = phi~ (1 + 2^-20), phi~ the evaluation)
            R = 2.0 ** -20
            err = np.abs(hi[fin0] / (1.0 + R) / pa[fin0] - 1.0)
            k = int(np.argmax(err))
            print(f"phi form {which}: max relative evaluation error {err[k]:.3g} at x = {a[fin0][k]:.6g} "
                  f"({err[k] / R:.2f} of the allowance)")
            assert err[k] < 0.5 * R


def test_phi_pair_equals_scalar_forms(Q):
    """The packed evaluation the check phase uses (qkds::phi_pair: the input
    bound of one edge and the output bound of another in the two halves of the
    packed binary32 unit) is bit for bit phi_bounds + phi_bounds_out, so the
    certification of the scalar forms (the sweep above, the exhaustive sweep in
    test_spec_bounds.py) carries over."""
    rng = np.random.default_rng(11)
    n = 1 << 20
    a = np.exp(rng.uniform(np.log(1e-30), np.log(120.0), n)).astype(np.float32)
    b = np.maximum(a, (a * (1.0 + rng.choice([0.0, 1e-6, 1e-3, 0.3], n))).astype(np.float32))
    s_lo = np.exp(rng.uniform(np.log(1e-12), np.log(900.0), n)).astype(np.float32)
    s_lo[rng.random(n) < 0.05] = 0.0                  # a widened sum that reached zero
    s_hi = np.maximum(s_lo, (s_lo * (1.0 + rng.choice([0.0, 1e-6, 1e-3, 0.3], n)) + 1e-14).astype(np.float32))
    # special points: the branch edges of phi_core and the clamps
    a[:8] = [0.35, 1.0, 80.0, 120.0, 1e-30, 2.0, np.nextafter(np.float32(0.35), 0), np.nextafter(np.float32(1), 0)]
    b[:8] = np.maximum(a[:8], b[:8])
    x = np.stack([a, b, s_lo, s_hi], axis=1).astype(np.float64).ravel()
    dx = torch.from_numpy(x).cuda()
    out = {}
    for which in (8, 9):
        dy = torch.empty_like(dx)
        Q._native.check(Q._native.lib().qkd_debug_math(which, dx.data_ptr(), dy.data_ptr(), dx.numel(), None))
        torch.cuda.synchronize()
        out[which] = dy.cpu().numpy().astype(np.float32).view(np.uint32)
    bad = np.nonzero(out[8] != out[9])[0]
    assert bad.size == 0, (bad[:8], x[bad[:8]], out[8][bad[:8]], out[9][bad[:8]])


def _intervals(rng, n, lo_exp, hi_exp, zero_share):
    lo = np.exp(rng.uniform(np.log(lo_exp), np.log(hi_exp), n)).astype(np.float32)
    lo[rng.random(n) < zero_share] = 0.0
    hi = np.maximum(lo, (lo * (1.0 + rng.choice([0.0, 1e-6, 1e-3, 0.3], n)) + 1e-14).astype(np.float32))
    return lo, hi


@pytest.mark.parametrize("packed,scalar,edges", [
    (14, 15, [0.0, 1e-30, 0.35, 1.0, 2.0, 80.0, 120.0, np.inf]),      # input form (kPhiHuge = 80)
    (16, 17, [0.0, 1e-12, 0.5, 1.0 / np.log(2), 115.0, 900.0, np.inf]),  # output form (kPsiHuge = 115)
])
def test_packed_phi_bounds_equal_scalar(Q, packed, scalar, edges):
    """The interleaved decoder's packed bound forms (qkds::phi_bounds2 and
    phi_bounds_out2, decode_ilv.hip's check phase) are bit for bit two scalar
    phi_bounds / phi_bounds_out, whose soundness the sweeps above establish:
    1M random interval pairs plus every pair of the forms' branch edges (zero,
    the clamps kPhiHuge / kPsiHuge, +inf, the x = 1 switch)."""
    rng = np.random.default_rng(29 + packed)
    n = 1 << 20
    alo, ahi = _intervals(rng, n, 1e-30, 1000.0, 0.05)
    blo, bhi = _intervals(rng, n, 1e-30, 1000.0, 0.05)
    e = np.array(edges, np.float32)
    ea, eb = np.meshgrid(e, e)
    # degenerate intervals at the edges and intervals spanning neighbouring edges
    k = ea.size
    alo[:k], ahi[:k] = ea.ravel(), ea.ravel()
    blo[:k], bhi[:k] = eb.ravel(), np.maximum(eb.ravel(), np.roll(eb.ravel(), 1))
    x = np.stack([alo, ahi, blo, bhi], axis=1).astype(np.float64).ravel()
    dx = torch.from_numpy(x).cuda()
    out = {}
    for which in (packed, scalar):
        dy = torch.empty_like(dx)
        Q._native.check(Q._native.lib().qkd_debug_math(which, dx.data_ptr(), dy.data_ptr(), dx.numel(), None))
        torch.cuda.synchronize()
        out[which] = dy.cpu().numpy().astype(np.float32).view(np.uint32)
    bad = np.nonzero(out[packed] != out[scalar])[0]
    assert bad.size == 0, (bad[:8], x[bad[:8]], out[packed][bad[:8]], out[scalar][bad[:8]])


def test_phi_bounds_out_at_zero(Q):
    """A phi-domain sum that may be 0 (the reference's P / t can be exactly +-1)
    has an infinite upper bound."""
    a = np.array([0.0, 0.0, 1e-14], np.float64)
    b = np.array([1e-14, 3.0, 2e-14], np.float64)
    lo, hi = device_phi(Q, 5, psi_units(a, -1), psi_units(b, 1))
    assert np.isinf(hi[0]) and np.isinf(hi[1]) and np.isfinite(hi[2])
    assert (lo <= phi64(b)).all()


@pytest.mark.parametrize("cap", ["0", "1", "2", "3", "8", "50"])
def test_trials_config2_every_cap(Q, H, golden_vectors, monkeypatch, cap, qkd_opt):
    qkd_opt("QKD_SPEC_CAP", cap)
    seeds = seeds_dev(Q.make_seeds(777, 4096))
    ws = Q.Workspace(H)
    replays(Q, ws)
    r = Q.run_trials(H, seeds, 0.02, 0, 50, 100.0, True, workspace=ws)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == golden_vectors["c2_iters"]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == golden_vectors["c2_sp"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c2_ko"]).all()
    n = replays(Q, ws)
    print(f"cap {cap}: {n} of 4096 frames replayed exactly")
    if cap == "8":
        assert n < 4096 // 10          # the intervals certify almost every frame


@pytest.mark.parametrize("cap", ["2", "8", "50"])
def test_trials_config3_points_every_cap(Q, H, golden_vectors, monkeypatch, cap, qkd_opt):
    qkd_opt("QKD_SPEC_CAP", cap)
    seeds = seeds_dev(Q.make_seeds(777, 10000))
    ws = Q.Workspace(H)
    grid = golden_vectors["c3_qnom"]
    for s, qn in enumerate(grid):
        replays(Q, ws)
        r = Q.run_trials(H, seeds, float(qn), s, 50, 100.0, True, workspace=ws)
        torch.cuda.synchronize()
        assert (r.iterations.cpu().numpy() == golden_vectors["c3_iters"][s]).all(), (cap, s)
        assert (r.syndromes_match.cpu().numpy().astype(bool) == golden_vectors["c3_sp"][s]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c3_ko"][s]).all()
        print(f"cap {cap} q {qn:.2f}: {replays(Q, ws)} of 10000 replayed")


@pytest.mark.parametrize("q,max_it", [(0.05, 50), (0.09, 50), (0.11, 12), (0.15, 6)])
@pytest.mark.parametrize("thr", [100.0, 2.5, 0.7])
def test_spec_bits_match_oracle(Q, H, oracle_code, monkeypatch, q, max_it, thr, qkd_opt):
    """Decoded words of converging and failing frames (the cap at max_it lets the
    speculative iterations run to the end) equal the oracle's bit for bit."""
    qkd_opt("QKD_SPEC_CAP", "64")
    rng = np.random.default_rng(int(q * 1000) + int(thr * 10))
    f = 4
    alice = rng.integers(0, 2, (f, 10240))
    bob = alice ^ (rng.random((f, 10240)) < q)
    r = Q.qkd_ldpc(H, torch.from_numpy(alice.astype(np.uint8)).cuda(),
                   torch.from_numpy(bob.astype(np.uint8)).cuda(), q, max_it, thr, True, want_bits=True)
    torch.cuda.synchronize()
    its = r.iterations.cpu().numpy()
    sp = r.syndromes_match.cpu().numpy()
    ko = r.keys_match.cpu().numpy()
    bits = r.bits.cpu().numpy()
    for k in range(f):
        want = oracle_code.qkd_ldpc(alice[k], bob[k], q, max_it, thr, True)
        assert its[k] == want["iters"], (q, thr, k)
        assert bool(sp[k]) == want["sp_ok"] and bool(ko[k]) == want["key_ok"]
        assert (bits[k] == want["out"]).all(), (q, thr, k)


@pytest.mark.parametrize("cap", ["0", "8"])
@pytest.mark.parametrize("q", [0.02, 0.05])
def test_spec_llr_path_matches_oracle(Q, H, oracle_code, monkeypatch, cap, q, qkd_opt):
    """qkd_decode_batch (the reference's sum_product_decoding, LLR input) with
    the speculation on and off: decoded words, iteration counts and flags equal
    the oracle's; the LLR path has no folded first iteration, so the intervals
    start from the LLRs themselves."""
    qkd_opt("QKD_SPEC_CAP", cap)
    rng = np.random.default_rng(int(q * 1000))
    f = 24
    alice = rng.integers(0, 2, (f, 10240))
    bob = alice ^ (rng.random((f, 10240)) < q)
    lp = np.log((1 - q) / q)
    llr = np.where(bob == 1, -lp, lp) * (1.0 + 0.25 * rng.random((f, 10240)))   # not +-log_p only
    syn = np.stack([oracle_code.syndrome(a) for a in alice]).astype(np.uint8)
    ws = Q.Workspace(H)
    Q.spec_replays(ws, reset=True)
    r = Q.sum_product_decoding(H, torch.from_numpy(llr).cuda(), torch.from_numpy(syn).cuda(), 50, 100.0, True,
                               workspace=ws)
    torch.cuda.synchronize()
    bits = r.bits.cpu().numpy()
    its = r.iterations.cpu().numpy()
    ok = r.syndromes_match.cpu().numpy()
    for k in range(f):
        want = oracle_code.decode(llr[k], syn[k], 50, 100.0, True)
        assert its[k] == want["iters"], (cap, q, k)
        assert bool(ok[k]) == want["sp_ok"]
        assert (bits[k] == want["out"]).all(), (cap, q, k)
    print(f"LLR path cap {cap} q {q}: {Q.spec_replays(ws)} of {f} replayed")


def test_spec_policy_turns_off_at_high_qber(Q, H, golden_vectors, monkeypatch, qkd_opt):
    """At QBER 0.08 most frames cannot be certified: the first call replays
    many (the in-launch policy stops speculating after a sixth), later calls on
    the workspace skip the speculation for that QBER and up (QKD_CKPT_UNSAT=0:
    no checkpointed speculation either); the results are the golden ones
    throughout."""
    qkd_opt("QKD_SPEC_CAP", "8")
    qkd_opt("QKD_CKPT_UNSAT", "0")
    seeds = seeds_dev(Q.make_seeds(777, 10000))
    grid = golden_vectors["c3_qnom"]
    s = int(np.argmin(np.abs(grid - 0.08)))
    ws = Q.Workspace(H)
    counts = []
    for _ in range(3):
        Q.spec_replays(ws, reset=True)
        r = Q.run_trials(H, seeds, float(grid[s]), s, 50, 100.0, True, workspace=ws)
        torch.cuda.synchronize()
        assert (r.iterations.cpu().numpy() == golden_vectors["c3_iters"][s]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c3_ko"][s]).all()
        counts.append(Q.spec_replays(ws))
    print("replays per call at QBER 0.08:", counts)
    assert counts[0] > 0 and counts[-1] == 0


@pytest.mark.parametrize("trigger", ["16", "128", "1024"])
def test_ckpt_config3_points(Q, H, golden_vectors, monkeypatch, trigger, qkd_opt):
    """Checkpointed speculation (SPEC 2) forced at every config-3 point: exact
    iterations until fewer than `trigger` checks are unsatisfied, intervals
    from a saved message store, restores on failure (a trigger of 1024 makes
    most attempts fail and exercises the restores); golden results."""
    qkd_opt("QKD_SPEC_CAP", "8")
    qkd_opt("QKD_SPEC_CKPT", "1")
    qkd_opt("QKD_CKPT_UNSAT", trigger)
    seeds = seeds_dev(Q.make_seeds(777, 10000))
    ws = Q.Workspace(H)
    grid = golden_vectors["c3_qnom"]
    total = 0
    for s, qn in enumerate(grid):
        Q.spec_replays(ws, reset=True)
        r = Q.run_trials(H, seeds, float(qn), s, 50, 100.0, True, workspace=ws)
        torch.cuda.synchronize()
        assert (r.iterations.cpu().numpy() == golden_vectors["c3_iters"][s]).all(), (trigger, s)
        assert (r.syndromes_match.cpu().numpy().astype(bool) == golden_vectors["c3_sp"][s]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c3_ko"][s]).all()
        n = Q.spec_replays(ws)
        total += n
        print(f"trigger {trigger} q {qn:.2f}: {n} restores")
    if trigger == "1024":
        assert total > 0


@pytest.mark.parametrize("q,max_it,cap", [(0.07, 50, "8"), (0.09, 50, "64"), (0.11, 20, "64"), (0.08, 12, "3")])
def test_ckpt_bits_match_oracle(Q, H, oracle_code, monkeypatch, q, max_it, cap, qkd_opt):
    """Decoded words after checkpointed speculation (converging frames, frames
    that fail with the intervals running to max_it, caps that force restores)
    equal the oracle's bit for bit."""
    qkd_opt("QKD_SPEC_CAP", cap)
    qkd_opt("QKD_SPEC_CKPT", "1")
    qkd_opt("QKD_CKPT_UNSAT", "400")
    rng = np.random.default_rng(int(q * 1000) + max_it)
    f = 6
    alice = rng.integers(0, 2, (f, 10240))
    bob = alice ^ (rng.random((f, 10240)) < q)
    r = Q.qkd_ldpc(H, torch.from_numpy(alice.astype(np.uint8)).cuda(),
                   torch.from_numpy(bob.astype(np.uint8)).cuda(), q, max_it, 100.0, True, want_bits=True)
    torch.cuda.synchronize()
    its = r.iterations.cpu().numpy()
    bits = r.bits.cpu().numpy()
    for k in range(f):
        want = oracle_code.qkd_ldpc(alice[k], bob[k], q, max_it, 100.0, True)
        assert its[k] == want["iters"], (q, k)
        assert bool(r.syndromes_match[k]) == want["sp_ok"] and bool(r.keys_match[k]) == want["key_ok"]
        assert (bits[k] == want["out"]).all(), (q, k)


def test_ckpt_policy_default(Q, H, golden_vectors, monkeypatch, qkd_opt):
    """Default policy at QBER 0.07: the first call speculates from the first
    iteration and replays too many frames; the next calls switch to the
    checkpointed speculation; golden results throughout."""
    qkd_opt("QKD_SPEC_CAP", None)
    qkd_opt("QKD_CKPT_UNSAT", None)
    qkd_opt("QKD_SPEC_CKPT", None)
    seeds = seeds_dev(Q.make_seeds(777, 10000))
    grid = golden_vectors["c3_qnom"]
    s = int(np.argmin(np.abs(grid - 0.07)))
    ws = Q.Workspace(H)
    for _ in range(3):
        r = Q.run_trials(H, seeds, float(grid[s]), s, 50, 100.0, True, workspace=ws)
        torch.cuda.synchronize()
        assert (r.iterations.cpu().numpy() == golden_vectors["c3_iters"][s]).all()
        assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c3_ko"][s]).all()


# ---- certification: exhaustive bounds, fresh frames --------------------------------

F32_80 = int(np.float32(80.0).view(np.uint32))      # qkds::kPhiHuge
F32_115 = int(np.float32(115.0).view(np.uint32))    # qkds::kPsiHuge


@pytest.mark.parametrize("which,last", [(4, F32_80), (5, F32_115)])
def test_phi_bounds_exhaustive(Q, which, last):
    """EVERY positive binary32 argument up to the clamp (subnormals included, about
    1.1e9 points per form): the upper bound is >= phi, the lower bound <= phi, and the
    slope bound (with half its 2^-20 margin left for the tangent's own roundings) is
    >= |phi'|, against binary64 phi on the device. With these, the bounds over any
    [a, b] follow from phi's monotonicity and convexity (qkd_spec.h)."""
    res = (C.c_uint64 * 8)()
    Q._native.check(Q._native.lib().qkd_debug_phi_sweep(which, 1, last, res))
    pts, bad_hi, bad_lo, bad_sl = res[0], res[1], res[2], res[3]
    e_max = float(np.uint32(res[4]).view(np.float32))
    s_max = float(np.uint32(res[5]).view(np.float32))
    e_at = float(np.uint32(res[6]).view(np.float32))
    s_at = float(np.uint32(res[7]).view(np.float32))
    print(f"form {which}: {pts} points; violations hi {bad_hi} lo {bad_lo} slope {bad_sl}; "
          f"max evaluation error {e_max:.3f} of 2^-20 at {e_at:.6g}; "
          f"max |phi'| / slope bound {s_max:.6f} at {s_at:.6g}")
    assert pts == last
    assert bad_hi == 0 and bad_lo == 0 and bad_sl == 0
    assert e_max < 0.75
    assert s_max <= 1.0 + 2.0 ** -21          # the slope bound's own margin is 2^-20


FRESH = 100_000


@pytest.fixture(scope="module")
def fresh_seeds(Q):
    """Seeds beyond the golden vectors' first 10,000 (same stream, seed 777)."""
    return seeds_dev(Q.make_seeds(777, 10_000 + FRESH)[10_000:])


@pytest.mark.parametrize("q", [0.02, 0.03, 0.04, 0.05, 0.06, 0.07, 0.08])
def test_spec_matches_exact_on_fresh_frames(Q, H, fresh_seeds, monkeypatch, q, qkd_opt):
    """100,000 frames per QBER point that no golden vector covers: the default
    (speculative, policy-driven, run twice so the per-workspace policy settles and
    both of its modes run) against the exact iterations alone (QKD_SPEC_CAP=0):
    decoded words, iteration counts and flags identical."""
    ws = Q.Workspace(H)
    alice, bob, _ = Q.keygen(H, fresh_seeds, q, 0, workspace=ws)
    qkd_opt("QKD_SPEC_CAP", "0")
    ex = Q.qkd_ldpc(H, alice, bob, q, 50, 100.0, True, want_bits=True, workspace=ws)
    qkd_opt("QKD_SPEC_CAP", None)
    ws2 = Q.Workspace(H)
    Q.spec_replays(ws2, reset=True)
    for rep in range(2):
        sp = Q.qkd_ldpc(H, alice, bob, q, 50, 100.0, True, want_bits=True, workspace=ws2)
        torch.cuda.synchronize()
        n = Q.spec_replays(ws2, reset=True)
        assert torch.equal(sp.iterations, ex.iterations), (q, rep)
        assert torch.equal(sp.syndromes_match, ex.syndromes_match)
        assert torch.equal(sp.keys_match, ex.keys_match)
        assert torch.equal(sp.bits, ex.bits), (q, rep)
        print(f"q {q} pass {rep}: {FRESH} frames identical, {n} replayed exactly, "
              f"mean it {ex.iterations.double().mean().item():.3f}")


@pytest.mark.parametrize("q", [0.02, 0.04, 0.06])
def test_fold_table_equals_per_bit_form(Q, H, fresh_seeds, monkeypatch, q, qkd_opt):
    """The speculative kernel's folded first iteration from its per-pattern table
    (fold_table_fill) against the per-bit form (QKD_FOLD_TABLE=0): the same psi
    bounds give the same certified rounds, so outputs AND the count of frames the
    intervals could not certify agree. (The in-launch replay policy decides
    over frame-index windows, so which frames it keeps off the speculation does
    not depend on how fast either form runs.)"""
    seeds = fresh_seeds[:20_000]
    out = {}
    for tab in ("0", "1"):
        qkd_opt("QKD_FOLD_TABLE", tab)
        ws = Q.Workspace(H)
        alice, bob, _ = Q.keygen(H, seeds, q, 0, workspace=ws)
        Q.spec_replays(ws, reset=True)
        r = Q.qkd_ldpc(H, alice, bob, q, 50, 100.0, True, want_bits=True, workspace=ws)
        torch.cuda.synchronize()
        out[tab] = (r, Q.spec_replays(ws))
    (a, na), (b, nb) = out["0"], out["1"]
    assert torch.equal(a.iterations, b.iterations) and torch.equal(a.bits, b.bits)
    assert torch.equal(a.keys_match, b.keys_match) and torch.equal(a.syndromes_match, b.syndromes_match)
    assert na == nb, (q, na, nb)


@pytest.mark.parametrize("q", [0.02, 0.05])
def test_spec_llr_path_matches_exact_on_fresh_frames(Q, H, fresh_seeds, monkeypatch, q, qkd_opt):
    """The LLR entry (sum_product_decoding) on 100,000 fresh frames with LLRs that are
    not +-log_p (each scaled by 1 + U(0, 0.25)): speculative = exact."""
    ws = Q.Workspace(H)
    alice, bob, qx = Q.keygen(H, fresh_seeds, q, 0, workspace=ws)
    qq = float(qx[0].item())
    lp = float(np.log((1 - qq) / qq))
    g = torch.Generator(device="cuda").manual_seed(int(q * 1e4))
    scale = 1.0 + 0.25 * torch.rand(bob.shape, dtype=torch.float64, device="cuda", generator=g)
    llr = torch.where(bob == 1, -lp, lp) * scale
    syn = Q.calculate_syndrome(H, alice)
    qkd_opt("QKD_SPEC_CAP", "0")
    ex = Q.sum_product_decoding(H, llr, syn, 50, 100.0, True, workspace=ws)
    qkd_opt("QKD_SPEC_CAP", None)
    sp = Q.sum_product_decoding(H, llr, syn, 50, 100.0, True, workspace=Q.Workspace(H))
    torch.cuda.synchronize()
    assert torch.equal(sp.iterations, ex.iterations)
    assert torch.equal(sp.syndromes_match, ex.syndromes_match)
    assert torch.equal(sp.bits, ex.bits)


def test_psi_of_exact_pair_equals_scalar(Q):
    """The folded bit phase's packed psi bounds of two exact b2c (psi_of_exact2) equal
    the scalar psi_of_exact bit for bit, special values included (0, +-0, NaN, +-inf,
    the clamp, subnormal and tiny magnitudes, the branch edges)."""
    rng = np.random.default_rng(19)
    n = 1 << 20
    x = np.exp(rng.uniform(np.log(1e-35), np.log(150.0), n)) * rng.choice([-1.0, 1.0], n)
    special = np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 100.0, -100.0, 1e-30, -1e-30, 1e-31, 5e-324,
                        0.35, 1.0, 80.0, 2.0, -0.35, np.nextafter(0.35, 0), np.nextafter(1.0, 0)])
    x[: special.size] = special
    x[special.size: 2 * special.size] = special[::-1]
    dx = torch.from_numpy(x).cuda()
    out = {}
    for which in (10, 11):
        dy = torch.empty_like(dx)
        Q._native.check(Q._native.lib().qkd_debug_math(which, dx.data_ptr(), dy.data_ptr(), dx.numel(), None))
        torch.cuda.synchronize()
        out[which] = dy.cpu().numpy().view(np.uint64)
    bad = np.nonzero(out[10] != out[11])[0]
    assert bad.size == 0, (bad[:8], x[bad[:8]])


@pytest.mark.parametrize("q", [0.05, 0.08])
def test_replay_policy_independent_of_scheduling(Q, H, fresh_seeds, monkeypatch, q, qkd_opt):
    """The in-launch replay policy (decode_split.hip spec_policy) decides frame f from
    window f / 256 - 8 of the frame index, so the frames it keeps off the speculation,
    and with them the replay count, are the same whatever order the workgroups finish
    their frames in: a fresh workspace's first (speculative) call at a QBER where the
    policy turns the speculation off, run at the full grid and at 97 and 160
    workgroups (other completion orders), gives identical outputs AND replay counts."""
    seeds = fresh_seeds[:12_000]
    out = {}
    for grid in ("0", "97", "160"):
        if grid == "0":
            qkd_opt("QKD_DECODE_GRID", None)
        else:
            qkd_opt("QKD_DECODE_GRID", grid)
        ws = Q.Workspace(H)
        alice, bob, qx = Q.keygen(H, seeds, q, 0, workspace=ws)
        Q.spec_replays(ws, reset=True)
        r = Q.qkd_ldpc(H, alice, bob, float(qx[0].item()), 50, 100.0, True, want_bits=True, workspace=ws)
        torch.cuda.synchronize()
        out[grid] = (r, Q.spec_replays(ws))
        ws.close()
    (a, na) = out["0"]
    assert na > 0
    for g in ("97", "160"):
        b, nb = out[g]
        assert torch.equal(a.iterations, b.iterations) and torch.equal(a.bits, b.bits)
        assert torch.equal(a.keys_match, b.keys_match)
        assert na == nb, (q, g, na, nb)
