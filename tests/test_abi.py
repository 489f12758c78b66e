"""The C ABI library: loads, exports exactly what include/qkd_ldpc.h declares,
and its host-side logic (validation, readers, seeds, QBER grid) behaves like
the reference — all without touching a GPU."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT, write_alist

HEADER = os.path.join(ROOT, "include", "qkd_ldpc.h")


@pytest.fixture(scope="module")
def N():
    from qkd_ldpc_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        from qkd_ldpc_amd.build import build
        build()
    return _native


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qkd_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree(N):
    assert header_functions() == sorted(N.EXPORTS)


def test_library_exports_every_symbol(N):
    L = N.lib()
    for name in header_functions():
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(header_functions()) <= exported
    # nothing else of ours leaks out (hidden visibility)
    assert not [s for s in exported if s.startswith("_ZN3qkd")]


def test_abi_version_and_strings(N):
    L = N.lib()
    assert L.qkd_abi_version() == 1
    assert L.qkd_status_string(N.ERR_UNSORTED) == b"adjacency row not ascending"
    assert L.qkd_device_count() >= 0


def test_make_seeds_matches_oracle(N, oracle_mod):
    from qkd_ldpc_amd import make_seeds
    for s in (777, 0, 2**64 - 1, 123456789):
        assert (make_seeds(s, 64) == oracle_mod.seeds(s, 64)).all()


def test_qber_range_reference_rows():
    from qkd_ldpc_amd import qber_range
    # config 3 row: round(0.08 / 0.01) = 8 points, end exclusive
    g = qber_range(0.01, 0.09, 0.01)
    assert len(g) == 8 and g[0] == 0.01 and g[7] == 0.01 + 7 * 0.01
    # config.json row for R=0.489 -> code_rate 0.58: 0.06 .. 0.075 step 0.0005 = 30 points
    assert len(qber_range(0.06, 0.075, 0.0005)) == 30


def _create(N, n, m, ptr, idx):
    st = C.c_int(-1)
    p = np.ascontiguousarray(ptr, np.int32)
    i = np.ascontiguousarray(idx, np.int32)
    h = N.lib().qkd_code_create(n, m, p.ctypes.data, i.ctypes.data, 0, C.byref(st))
    if h:
        N.lib().qkd_code_destroy(h)
    return st.value, N.last_error()


def test_code_validation_statuses(N):
    # unsorted row -> the reference would mis-route messages silently (A1)
    st, msg = _create(N, 4, 2, [0, 2, 4], [1, 0, 2, 3])
    assert st == N.ERR_UNSORTED and "ascending" in msg
    st, _ = _create(N, 4, 2, [0, 2, 4], [0, 0, 2, 3])
    assert st == N.ERR_BAD_CODE                      # duplicate edge
    st, _ = _create(N, 4, 2, [0, 2, 4], [0, 9, 2, 3])
    assert st == N.ERR_BAD_CODE                      # out of range
    st, _ = _create(N, 4, 2, [1, 2, 4], [0, 1, 2, 3])
    assert st == N.ERR_BAD_CODE                      # check_ptr[0] != 0
    st, _ = _create(N, 0, 2, [0, 2, 4], [0, 1, 2, 3])
    assert st == N.ERR_INVALID_ARG
    st, _ = _create(N, 80, 1, [0, 65], list(range(65)))
    assert st == N.ERR_UNSUPPORTED                   # check degree > 64 (one wavefront)


def test_valid_code_without_gpu_reports_device_error(N):
    if N.lib().qkd_device_count() > 0:
        pytest.skip("a GPU is visible")
    st, msg = _create(N, 4, 2, [0, 2, 4], [0, 1, 2, 3])
    assert st == N.ERR_DEVICE and "device" in msg


def _alist_status(N, path):
    st = C.c_int(-1)
    h = N.lib().qkd_code_from_alist(path.encode(), 0, C.byref(st))
    if h:
        N.lib().qkd_code_destroy(h)
    return st.value, N.last_error()


def test_alist_reader_errors(N, tmp_path):
    st, msg = _alist_status(N, str(tmp_path / "missing.txt"))
    assert st == N.ERR_IO and "Failed to open file" in msg
    p = tmp_path / "bad.txt"
    p.write_text("4 2\n2 4 1\n")
    assert _alist_status(N, str(p))[0] == N.ERR_IO
    p.write_text("4 2\n1 2\n1 1 1 1\n2 2\n1\n1\n2\n2\n1 2\n3 4 9\n")
    st, msg = _alist_status(N, str(p))
    assert st == N.ERR_IO and "non-zero" in msg
    # bit rows listing checks out of order -> the reference would mis-route (A1)
    p.write_text("4 2\n2 4\n2 2 2 2\n4 4\n2 1\n1 2\n1 2\n1 2\n1 2 3 4\n1 2 3 4\n")
    st, msg = _alist_status(N, str(p))
    assert st == N.ERR_UNSORTED


def test_alist_reader_accepts_reference_layout(N, golden_code, tmp_path):
    """Zero-padded, 1-based rows as in alist_sparse_matrices/*.txt: parse succeeds up to
    the device step (CPU box) and yields the reference adjacency."""
    g = golden_code
    p = str(tmp_path / "c.alist")
    write_alist(p, 10240, 5231, g["bit_off"], g["bit_idx"], g["chk_off"], g["chk_idx"])
    st, msg = _alist_status(N, p)
    if N.lib().qkd_device_count() == 0:
        assert st == N.ERR_DEVICE, msg            # parsed + validated, then no device
    else:
        assert st == N.OK, msg


def _alist_status_ex(N, path, flags):
    st = C.c_int(-1)
    h = N.lib().qkd_code_from_alist_ex(path.encode(), 0, flags, C.byref(st))
    if h:
        N.lib().qkd_code_destroy(h)
    return st.value, N.last_error()


def _parsed(N, st):
    """Parsed and validated: OK with a GPU, the device error without one."""
    return st == (N.ERR_DEVICE if N.lib().qkd_device_count() == 0 else N.OK)


def test_alist_reader_sort_rows_option(N, tmp_path):
    """QKD_READ_SORT_ROWS reads a file whose lines are not ascending as the matrix it
    describes; without it the file is rejected (the reference mis-routes, A1)."""
    p = tmp_path / "u.txt"
    p.write_text("4 2\n2 4\n2 2 2 2\n4 4\n2 1\n1 2\n1 2\n1 2\n4 3 2 1\n1 2 3 4\n")
    assert _alist_status_ex(N, str(p), 0)[0] == N.ERR_UNSORTED
    st, msg = _alist_status_ex(N, str(p), N.READ_SORT_ROWS)
    assert _parsed(N, st), msg
    # sorting does not excuse a wrong edge set
    p.write_text("4 2\n2 4\n2 2 2 2\n4 4\n2 1\n1 2\n1 2\n1 1\n4 3 2 1\n1 2 3 4\n")
    assert _alist_status_ex(N, str(p), N.READ_SORT_ROWS)[0] == N.ERR_BAD_CODE
    assert _alist_status_ex(N, str(p), 0x80)[0] == N.ERR_INVALID_ARG


def test_alist_reader_line_endings_and_blank_tail(N, golden_code, tmp_path):
    """CRLF line endings and trailing blank lines (files edited on other systems)."""
    g = golden_code
    p = str(tmp_path / "c.alist")
    write_alist(p, 10240, 5231, g["bit_off"], g["bit_idx"], g["chk_off"], g["chk_idx"], pad=False)
    text = open(p).read().replace("\n", "\r\n") + "\r\n\r\n"
    with open(p, "w", newline="") as f:
        f.write(text)
    st, msg = _alist_status(N, p)
    assert _parsed(N, st), msg


def test_dense_reader_errors(N, tmp_path):
    def status(text):
        p = tmp_path / "d.txt"
        p.write_text(text)
        st = C.c_int(-1)
        h = N.lib().qkd_code_from_dense(str(p).encode(), 0, C.byref(st))
        if h:
            N.lib().qkd_code_destroy(h)
        return st.value, N.last_error()
    assert status("1 0 2\n0 1 1\n")[0] == N.ERR_IO          # value not 0/1
    assert status("1 0 1\n0 1\n")[0] == N.ERR_IO            # ragged rows
    st, msg = status("1 0 0\n1 1 0\n")
    assert st == N.ERR_IO and "Column '3'" in msg           # zero column
    st, msg = status("1 1 1\n0 0 0\n")
    assert st == N.ERR_IO and "Column" in msg or "Row" in msg


def test_library_reads_no_environment():
    """Product behaviour never depends on the process environment: neither the
    HIP library nor the compatibility shim imports getenv (debug and A/B
    options go through qkd_debug_set_option / qkd_amd_set_*)."""
    libs = [os.path.join(ROOT, "qkd_ldpc_amd", "lib", "libqkd_ldpc_amd.so")]
    shim = os.path.join(ROOT, "qkd_ldpc_amd", "lib", "libqkd_ldpc_compat.so")
    if os.path.exists(shim):
        libs.append(shim)
    for lib in libs:
        out = subprocess.check_output(["nm", "-D", "--undefined-only", lib], text=True)
        names = {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}
        assert not names & {"getenv", "secure_getenv", "__libc_secure_getenv"}, lib
    for dirpath, _, files in os.walk(os.path.join(ROOT, "qkd_ldpc_amd", "csrc")):
        for f in files:
            assert "getenv" not in open(os.path.join(dirpath, f), errors="replace").read(), f


def test_debug_options_validated(N):
    """qkd_debug_set_option: known names set and reset (process-wide, no device
    needed), unknown names are errors."""
    L = N.lib()
    assert L.qkd_debug_set_option(None, b"QKD_SPEC_CAP", b"3") == 0
    assert L.qkd_debug_set_option(None, b"QKD_SPEC_CAP", None) == 0
    assert L.qkd_debug_set_option(None, b"QKD_NO_SUCH_OPTION", b"1") != 0
    assert "unknown debug option" in N.last_error()
    assert L.qkd_debug_set_option(None, None, b"1") != 0


def test_product_never_imports_oracle():
    """The oracle is test infrastructure: no product source references it."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "qkd_ldpc_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".hpp")):
                text = open(os.path.join(dirpath, f), errors="replace").read()
                assert "oracle" not in text.lower() or f == "__init__.py" and "oracle" not in text, f


# ---- Python wrapper argument checks (the kernels read F x N / F x M elements) -------

def test_frames_rejects_ragged_and_short_buffers():
    import torch
    import qkd_ldpc_amd as Q
    assert Q._frames(torch.zeros(3, 10), 10, "llr") == 3
    assert Q._frames(torch.zeros(10), 10, "llr") == 1
    for bad in (torch.zeros(25), torch.zeros(3, 9), torch.zeros(2, 3, 10)):
        with pytest.raises(Q.QkdError):
            Q._frames(bad, 10, "llr")
    with pytest.raises(Q.QkdError):
        Q._frames(torch.zeros(2, 5), 5, "syndrome", frames=3)


def test_wrappers_reject_host_tensors():
    import torch
    import qkd_ldpc_amd as Q
    with pytest.raises(Q.QkdError):
        Q._need_cuda(torch.zeros(4, dtype=torch.float64), torch.float64, "llr")
    with pytest.raises(Q.QkdError):
        Q._need_cuda(np.zeros(4), torch.float64, "llr")


@pytest.mark.gpu
def test_wrappers_reject_mismatched_shapes(golden_code):
    import torch
    import qkd_ldpc_amd as Q
    g = golden_code
    H = Q.HMatrix.from_check_lists(10240, g["chk_off"], g["chk_idx"])
    llr = torch.zeros(4, 10240, dtype=torch.float64, device="cuda")
    syn = torch.zeros(4, 5231, dtype=torch.uint8, device="cuda")
    bits = torch.zeros(4, 10240, dtype=torch.uint8, device="cuda")
    cases = [
        lambda: Q.sum_product_decoding(H, llr, syn[:3]),                     # short syndrome
        lambda: Q.sum_product_decoding(H, llr.view(-1)[:-5], syn),           # not a multiple of N
        lambda: Q.sum_product_decoding(H, llr, syn.view(-1)[:4 * 5230]),     # flat, wrong width
        lambda: Q.qkd_ldpc(H, bits, bits[:2], 0.02),                          # bob shorter than alice
        lambda: Q.calculate_syndrome(H, bits[:, :100]),
        lambda: Q.keygen(H, torch.zeros(2, 2, dtype=torch.int64, device="cuda"), 0.02),
        lambda: Q.run_trials(H, torch.zeros(4, dtype=torch.int64, device="cuda"), 0.02,
                             out=Q.run_trials(H, torch.zeros(2, dtype=torch.int64, device="cuda"), 0.02)),
    ]
    for k, call in enumerate(cases):
        with pytest.raises(Q.QkdError):
            call()
    torch.cuda.synchronize()
