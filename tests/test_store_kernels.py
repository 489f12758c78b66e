"""The two message-store kernels behind the same C ABI.

The sum-product rules run on decode_split_kernel (decode_split.hip: message
slots split between LDS and global memory, bit totals in registers) by
default; QKD_DECODE_KERNEL=classic selects decode_kernel (decode.hip: the
classic bit-major c2b store with LDS bit totals). Both must give the oracle's
results bit for bit (binary64), and the binary32 variant must give the same
bits on both (the same binary32 operations in the same order).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_gpu_parity import _qkd_both, decode_both, dev, llr_of, seeds_dev  # noqa: E402

KERNELS = ["split", "classic"]


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


def _use(qkd_opt, kernel):
    if kernel == "classic":
        qkd_opt("QKD_DECODE_KERNEL", "classic")
    else:
        qkd_opt("QKD_DECODE_KERNEL", None)


@pytest.mark.parametrize("kernel", KERNELS)
def test_trials_config2_golden(Q, H, golden_vectors, monkeypatch, kernel, qkd_opt):
    _use(qkd_opt, kernel)
    r = Q.run_trials(H, seeds_dev(Q.make_seeds(777, 4096)), 0.02, 0, 50, 100.0, True)
    torch.cuda.synchronize()
    assert (r.iterations.cpu().numpy() == golden_vectors["c2_iters"]).all()
    assert (r.keys_match.cpu().numpy().astype(bool) == golden_vectors["c2_ko"]).all()


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("thr,thr_on,max_it", [(100.0, True, 50), (100.0, False, 50), (0.5, True, 7),
                                               (100.0, True, 1), (100.0, True, 2)])
def test_llr_path(Q, H, oracle_code, oracle_mod, monkeypatch, kernel, thr, thr_on, max_it, qkd_opt):
    _use(qkd_opt, kernel)
    seeds = oracle_mod.seeds(99, 6)
    llr, syn = [], []
    for s in seeds:
        a, b, q = oracle_mod.keygen(int(s), 10240, 0.06)
        llr.append(llr_of(b, q))
        syn.append(oracle_code.syndrome(a))
    decode_both(Q, H, oracle_code, np.stack(llr), np.stack(syn), max_it, thr, thr_on)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("q,max_it", [(0.03, 50), (0.5, 6), (0.7, 4), (0.05, 1), (0.05, 2)])
def test_keys_path_tables(Q, H, oracle_code, monkeypatch, kernel, q, max_it, qkd_opt):
    _use(qkd_opt, kernel)
    rng = np.random.default_rng(int(q * 100) + max_it)
    alice = rng.integers(0, 2, (3, 10240))
    bob = alice ^ (rng.random((3, 10240)) < min(q, 0.3))
    _qkd_both(Q, H, oracle_code, alice, bob, q, max_it, 100.0, True)


@pytest.mark.parametrize("q", [0.05, 0.08])
def test_sp_f32_same_bits_on_both_kernels(Q, H, monkeypatch, q, qkd_opt):
    seeds = seeds_dev(Q.make_seeds(31, 64))
    out = {}
    for kernel in KERNELS:
        _use(qkd_opt, kernel)
        r = Q.run_trials(H, seeds, q, 0, 50, 100.0, True, variant="sp_f32")
        a, b, qq = Q.keygen(H, seeds, q)
        rb = Q.qkd_ldpc(H, a, b, float(qq[0]), 50, 100.0, True, want_bits=True, variant="sp_f32")
        torch.cuda.synchronize()
        out[kernel] = (r.iterations.cpu().numpy(), r.keys_match.cpu().numpy(), rb.bits.cpu().numpy())
    for x, y in zip(out["split"], out["classic"]):
        assert (x == y).all()


def test_split_kernel_is_default_and_classic_selectable(Q, H, monkeypatch, qkd_opt):
    """Both selections run (QKD_PHASE_TIMING off): equal per-frame results on a
    QBER point where frames need many iterations."""
    seeds = seeds_dev(Q.make_seeds(5, 256))
    res = {}
    for kernel in KERNELS:
        _use(qkd_opt, kernel)
        r = Q.run_trials(H, seeds, 0.075, 0, 50, 100.0, True)
        torch.cuda.synchronize()
        res[kernel] = r.iterations.cpu().numpy()
    assert (res["split"] == res["classic"]).all()
    assert res["split"].mean() > 10
