"""Codes longer than the LDS-resident totals allow (N > 20480). The reference's
binary64 rule runs in the split-store kernel (decode_split.hip: a share of the
message slots in LDS, the rest in the workgroup's global region, up to N =
65536), speculative interval iterations included; the classic kernel with its
bit totals in global scratch (decode_kernel<..., GT = true>) stays behind
QKD_DECODE_KERNEL=classic and for longer codes. Random regular (3, 6) codes;
parity with the oracle bit for bit for both kernels, fused trials included
(both key generators: the jump-ahead one for floor(N q) <= 4096 and the serial
one beyond)."""
import numpy as np
import pytest

from conftest import write_alist


def regular_code(n, dv=3, dc=6, seed=0):
    """Random (dv, dc)-regular parity-check matrix without repeated edges, as
    check rows (ascending) -> (check_ptr, check_idx)."""
    rng = np.random.default_rng(seed)
    m = n * dv // dc
    while True:
        sockets = np.repeat(np.arange(n), dv)
        rng.shuffle(sockets)
        rows = sockets.reshape(m, dc)
        srt = np.sort(rows, axis=1)
        bad = (np.diff(srt, axis=1) == 0).any(axis=1)
        if not bad.any():
            break
        # repair: re-shuffle only the rows with a repeated bit (rare)
        for _ in range(100):
            idx = np.nonzero(bad)[0]
            if idx.size == 0:
                break
            pool = np.concatenate([rows[idx].ravel(), rows[rng.integers(0, m, idx.size)].ravel()])
            rng.shuffle(pool)
            rows[idx] = pool[: idx.size * dc].reshape(idx.size, dc)
            srt = np.sort(rows, axis=1)
            bad = (np.diff(srt, axis=1) == 0).any(axis=1)
        if not bad.any() and np.bincount(rows.ravel(), minlength=n).max() == dv:
            break
    rows = np.sort(rows, axis=1)
    return m, np.arange(0, m * dc + 1, dc, dtype=np.int32), rows.ravel().astype(np.int32)


@pytest.fixture(scope="module")
def big():
    n = 40000
    m, cp, ci = regular_code(n, seed=11)
    return n, m, cp, ci


def test_large_code_parses_and_validates(big):
    """CPU side: creation reaches the device step (no size limit below the plan's)."""
    import ctypes as C
    from qkd_ldpc_amd import _native as N
    n, m, cp, ci = big
    st = C.c_int(-1)
    h = N.lib().qkd_code_create(n, m, cp.ctypes.data, ci.ctypes.data, 0, C.byref(st))
    if h:
        N.lib().qkd_code_destroy(h)
    assert st.value == (N.ERR_DEVICE if N.lib().qkd_device_count() == 0 else N.OK), N.last_error()


torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def Q():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import qkd_ldpc_amd as Q
    return Q


@pytest.fixture(scope="module")
def big_codes(big, Q, oracle_mod, tmp_path_factory):
    n, m, cp, ci = big
    H = Q.HMatrix.from_check_lists(n, cp, ci)
    cptr, cidx, bptr, bidx = H.adjacency()
    p = str(tmp_path_factory.mktemp("big") / "big.alist")
    write_alist(p, n, m, bptr, bidx, cptr, cidx)
    return H, oracle_mod.Code.from_alist(p)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["split", "classic"])
@pytest.mark.parametrize("q,thr,thr_on", [(0.03, 100.0, True), (0.06, 2.5, True), (0.04, 0.0, False)])
def test_large_code_decode_bit_exact(Q, big_codes, oracle_mod, monkeypatch, kernel, q, thr, thr_on, qkd_opt):
    if kernel == "classic":
        qkd_opt("QKD_DECODE_KERNEL", "classic")
    H, oc = big_codes
    n = H.num_bit_nodes
    frames = []
    for s in oracle_mod.seeds(99, 6):
        a, b, qq = oracle_mod.keygen(int(s), n, q)
        lp = np.log((1 - qq) / qq)
        frames.append((np.where(b == 1, -lp, lp), oc.syndrome(a)))
    llr = np.stack([f[0] for f in frames])
    syn = np.stack([f[1] for f in frames]).astype(np.uint8)
    r = Q.sum_product_decoding(H, torch.from_numpy(llr).cuda(), torch.from_numpy(syn).cuda(), 40,
                               thr if thr_on else 100.0, thr_on)
    torch.cuda.synchronize()
    for f in range(len(frames)):
        want = oc.decode(llr[f], syn[f], 40, thr, thr_on)
        assert int(r.iterations[f]) == want["iters"]
        assert bool(r.syndromes_match[f]) == want["sp_ok"]
        assert (r.bits[f].cpu().numpy() == want["out"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["split", "classic"])
@pytest.mark.parametrize("q", [0.03, 0.05, 0.11])
def test_large_code_trials_equal_oracle(Q, big_codes, oracle_mod, monkeypatch, kernel, q, qkd_opt):
    """Fused trials (keygen + decode + compare); at q = 0.11 floor(N q) = 4400
    flips take the serial key generator."""
    if kernel == "classic":
        qkd_opt("QKD_DECODE_KERNEL", "classic")
    H, oc = big_codes
    seeds = oracle_mod.seeds(777, 8)
    r = Q.run_trials(H, torch.from_numpy(seeds.view(np.int64)).cuda(), q, 0, 40)
    torch.cuda.synchronize()
    want = oc.trials(q, seeds, 0, 40, 100.0, True)
    assert (r.iterations.cpu().numpy() == want["iters"]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == want["sp_ok"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == want["key_ok"]).all()
    assert (r.exact_qber.cpu().numpy() == want["exact_q"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sp_f32", "minsum"])
def test_large_code_variants_decode(Q, big_codes, variant):
    H, _ = big_codes
    seeds = torch.from_numpy(Q.make_seeds(5, 64).view(np.int64)).cuda()
    r = Q.run_trials(H, seeds, 0.02, 0, 40, variant=variant)
    torch.cuda.synchronize()
    assert r.syndromes_match.cpu().numpy().all() and r.keys_match.cpu().numpy().all()


@pytest.mark.gpu
@pytest.mark.parametrize("dv,dc,n", [(3, 6, 2400), (3, 12, 2400), (2, 16, 2400), (3, 6, 2460)])
def test_frame_syn_sliced_equals_plain(monkeypatch, dv, dc, n, qkd_opt):
    """frame_syn_sliced_kernel (frames bit-sliced, uint16 check rows of width
    8 or 16) against frame_syn_kernel (QKD_SYN_SLICED=0): the
    same decoded words, iterations and flags on the keys path."""
    import torch
    import qkd_ldpc_amd as Q
    # (N = 2460: an odd number of key words, the last slice pair half empty)
    m, cp, ci = regular_code(n, dv, dc, seed=dc)
    H = Q.HMatrix.from_check_lists(n, cp, ci)
    seeds = torch.from_numpy(Q.make_seeds(99, 600).view(np.int64)).cuda()
    a, b, q = Q.keygen(H, seeds, 0.01)
    out = {}
    for mode in ("1", "0"):
        qkd_opt("QKD_SYN_SLICED", mode)
        r = Q.qkd_ldpc(H, a, b, float(q[0]), 50, 100.0, True, want_bits=True)
        torch.cuda.synchronize()
        out[mode] = r
    x, y = out["1"], out["0"]
    assert torch.equal(x.iterations, y.iterations) and torch.equal(x.bits, y.bits)
    assert torch.equal(x.keys_match, y.keys_match) and torch.equal(x.syndromes_match, y.syndromes_match)


@pytest.mark.gpu
@pytest.mark.parametrize("q,grid", [(0.03, 1), (0.05, 2), (0.08, 3)])
def test_interleaved_trials_equal_oracle(Q, big_codes, oracle_mod, monkeypatch, q, grid, qkd_opt):
    """The frame-interleaved decoder (decode_ilv.hip, forced with QKD_ILV=1)
    against the oracle: 40 frames through 1-3 workgroups, so columns take
    several frames each (the queue refill); at q = 0.08 frames hand off to the
    split kernel's exact replays."""
    qkd_opt("QKD_ILV", "1")
    qkd_opt("QKD_ILV_GRID", str(grid))
    H, oc = big_codes
    seeds = oracle_mod.seeds(123, 40)
    r = Q.run_trials(H, torch.from_numpy(seeds.view(np.int64)).cuda(), q, 0, 40)
    torch.cuda.synchronize()
    want = oc.trials(q, seeds, 0, 40, 100.0, True)
    assert (r.iterations.cpu().numpy() == want["iters"]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == want["sp_ok"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == want["key_ok"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("q,cap,frames", [(0.02, None, 4096), (0.03, None, 4096), (0.03, "2", 4096),
                                          (0.05, None, 4096), (0.04, None, 10000)])
def test_interleaved_equals_split_at_scale(Q, big_codes, monkeypatch, q, cap, frames, qkd_opt):
    """4096 frames: the interleaved decoder (its default for this code at this
    batch size) and the split kernel (QKD_ILV=0) give the same iterations,
    syndrome and key flags. QKD_SPEC_CAP=2 hands every frame still iterating
    after two interval rounds to the split kernel (its frame-list path);
    10,000 frames take the columns through two to three frames each."""
    H, _ = big_codes
    if cap:
        qkd_opt("QKD_SPEC_CAP", cap)
    seeds = torch.from_numpy(Q.make_seeds(2024, frames).view(np.int64)).cuda()
    a, b, qq = Q.keygen(H, seeds, q)
    out = {}
    for mode in ("1", "0"):
        qkd_opt("QKD_ILV", mode)
        r = Q.qkd_ldpc(H, a, b, float(qq[0]), 50)
        torch.cuda.synchronize()
        out[mode] = r
    x, y = out["1"], out["0"]
    assert torch.equal(x.iterations, y.iterations)
    assert torch.equal(x.syndromes_match, y.syndromes_match) and torch.equal(x.keys_match, y.keys_match)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [0.02, 0.04])
def test_interleaved_global_targets_equal_split(Q, monkeypatch, q, qkd_opt):
    """N = 60,000 (M = 30,000): the interleaved decoder's three LDS syndrome
    arrays would not fit, so its target syndrome words live in global memory
    (decode_ilv_kernel<..., TG = true>); 1024 frames give the same iterations,
    syndrome and key flags as the split kernel (QKD_ILV=0)."""
    n = 60000
    m, cp, ci = regular_code(n, seed=11)
    H = Q.HMatrix.from_check_lists(n, cp, ci)
    seeds = torch.from_numpy(Q.make_seeds(2024, 1024).view(np.int64)).cuda()
    a, b, qq = Q.keygen(H, seeds, q)
    out = {}
    for mode in ("1", "0"):
        qkd_opt("QKD_ILV", mode)
        r = Q.qkd_ldpc(H, a, b, float(qq[0]), 50)
        torch.cuda.synchronize()
        out[mode] = r
    x, y = out["1"], out["0"]
    assert torch.equal(x.iterations, y.iterations)
    assert torch.equal(x.syndromes_match, y.syndromes_match) and torch.equal(x.keys_match, y.keys_match)


@pytest.fixture(scope="module", params=[70002, 80002, 131070])
def long_codes(request, Q, oracle_mod, tmp_path_factory):
    """Codes past kMaxBitsSplit (65,536 bits): N = 70,002 (M = 35,001, the
    interleaved decoder's target syndrome words in global memory), 80,002
    (M = 40,001: its uncertainty words there too, decode_ilv_kernel<..., UG>)
    and 131,070 (M = 65,535: the largest the long-code path takes,
    kMaxBitsSplitLong / kMaxChecksSplit); N mod 64 != 0 (a ragged last key
    word)."""
    n = request.param
    m, cp, ci = regular_code(n, seed=5)
    H = Q.HMatrix.from_check_lists(n, cp, ci)
    cptr, cidx, bptr, bidx = H.adjacency()
    p = str(tmp_path_factory.mktemp("long") / f"long{n}.alist")
    write_alist(p, n, m, bptr, bidx, cptr, cidx)
    return H, oracle_mod.Code.from_alist(p)


@pytest.mark.gpu
@pytest.mark.parametrize("ilv,q,cap", [("1", 0.03, None), ("1", 0.07, None), ("1", 0.05, "2"), ("0", 0.04, None)])
def test_long_code_trials_equal_oracle(Q, long_codes, oracle_mod, ilv, q, cap, qkd_opt):
    """Long codes on the keys path: the interleaved decoder (QKD_ILV=1, two
    workgroups so columns refill) with its uncertified frames handed to the
    exact long-code split kernel (decode_split_kernel<..., LONG = true>; q =
    0.07 and QKD_SPEC_CAP=2 hand many off), and the classic kernel
    (QKD_ILV=0), against the oracle bit for bit."""
    qkd_opt("QKD_ILV", ilv)
    qkd_opt("QKD_ILV_GRID", "2")
    if cap:
        qkd_opt("QKD_SPEC_CAP", cap)
    H, oc = long_codes
    seeds = oracle_mod.seeds(4242, 24)
    r = Q.run_trials(H, torch.from_numpy(seeds.view(np.int64)).cuda(), q, 0, 40)
    torch.cuda.synchronize()
    want = oc.trials(q, seeds, 0, 40, 100.0, True)
    assert (r.iterations.cpu().numpy() == want["iters"]).all()
    assert (r.syndromes_match.cpu().numpy().astype(bool) == want["sp_ok"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == want["key_ok"]).all()
    assert (r.exact_qber.cpu().numpy() == want["exact_q"]).all()


@pytest.mark.gpu
def test_long_code_handoffs_counted(Q, long_codes, qkd_opt):
    """QKD_SPEC_CAP=1: every frame still iterating after its first interval
    round goes to the long-code split kernel; the replay counter counts them."""
    qkd_opt("QKD_ILV", "1")
    qkd_opt("QKD_SPEC_CAP", "1")
    H, _ = long_codes
    seeds = torch.from_numpy(Q.make_seeds(31, 256).view(np.int64)).cuda()
    ws = Q.Workspace(H)
    a, b, qq = Q.keygen(H, seeds, 0.03)
    r = Q.qkd_ldpc(H, a, b, float(qq[0]), 50, workspace=ws)
    torch.cuda.synchronize()
    assert Q.spec_replays(ws) > 0
    assert r.keys_match.cpu().numpy().all()
