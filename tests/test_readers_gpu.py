"""Reader hardening on the device path: a file whose lines are shuffled, read with
QKD_READ_SORT_ROWS, decodes exactly like the canonical file (same code object)."""
import numpy as np
import pytest

from conftest import write_alist

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def test_sorted_read_equals_canonical(golden_code, tmp_path):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    import qkd_ldpc_amd as Q
    g = golden_code
    canon = str(tmp_path / "canon.alist")
    write_alist(canon, 10240, 5231, g["bit_off"], g["bit_idx"], g["chk_off"], g["chk_idx"])
    # same matrix, every line's entries reversed
    rng = np.random.default_rng(3)
    bo, bi, co, ci = (np.array(g[k]) for k in ("bit_off", "bit_idx", "chk_off", "chk_idx"))
    bi2, ci2 = bi.copy(), ci.copy()
    for i in range(10240):
        bi2[bo[i]:bo[i + 1]] = rng.permutation(bi[bo[i]:bo[i + 1]])
    for j in range(5231):
        ci2[co[j]:co[j + 1]] = rng.permutation(ci[co[j]:co[j + 1]])
    shuf = str(tmp_path / "shuf.alist")
    write_alist(shuf, 10240, 5231, bo, bi2, co, ci2)
    with pytest.raises(Q.QkdError):
        Q.HMatrix.from_alist(shuf)
    A = Q.HMatrix.from_alist(canon)
    B = Q.HMatrix.from_alist(shuf, sort_rows=True)
    for x, y in zip(A.adjacency(), B.adjacency()):
        assert (x == y).all()
    seeds = torch.from_numpy(Q.make_seeds(777, 512).view(np.int64)).cuda()
    ra = Q.run_trials(A, seeds, 0.06)
    rb = Q.run_trials(B, seeds, 0.06)
    torch.cuda.synchronize()
    assert (ra.iterations.cpu() == rb.iterations.cpu()).all()
    assert (ra.keys_match.cpu() == rb.keys_match.cpu()).all()
