"""qkd_ldpc_amd — MI355X-native QKD LDPC sum-product decoding.

Python view of the C ABI (include/qkd_ldpc.h). It mirrors the reference's
hot-path interface (ColdCloudd/QKD_LDPC, src/qkd_ldpc_algorithm.hpp and
src/array_and_matrix_operations.hpp) with batched, device-resident arrays:

  reference (one frame, host int arrays)         here (F frames, torch tensors on the GPU)
  ---------------------------------------------  ------------------------------------------
  H_matrix + read_sparse_alist_matrix             HMatrix.from_alist(path)
  read_dense_matrix                               HMatrix.from_dense(path)
  calculate_syndrome_irregular/_regular           calculate_syndrome(H, bits)
  sum_product_decoding_irregular/_regular         sum_product_decoding(H, llr, syndrome, ...)
  QKD_LDPC_irregular/_regular                     qkd_ldpc(H, alice, bob, qber, ...)
  generate_random_bit_array + introduce_errors    keygen(H, seeds, q_nominal, ...)
  run_trial over a batch + the batch reduction    run_trials(H, seeds, q_nominal, ...)
  seeds of QKD_LDPC_batch_simulation              make_seeds(simulation_seed, count)
  get_rate_based_QBER_range (one table row)       qber_range(begin, end, step)
  QKD_LDPC_interactive_simulation                 interactive_simulation(H, seed, qbers, ...)

Errors surface as QkdError (a RuntimeError, as the reference throws
std::runtime_error). Every call runs HIP kernels; nothing falls back to CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N
from ._native import FLAG_THRESHOLD, QkdError

try:
    import torch
except Exception:  # pragma: no cover
    torch = None

__all__ = [
    "HMatrix", "QkdError", "calculate_syndrome", "sum_product_decoding",
    "sum_product_decoding_irregular", "sum_product_decoding_regular", "qkd_ldpc",
    "QKD_LDPC_irregular", "QKD_LDPC_regular", "keygen", "run_trials", "make_seeds",
    "qber_range", "Workspace", "counters_to_stats", "decoder_flags", "trace_decode", "set_debug_option",
    "spec_replays", "interactive_simulation",
]


def decoder_flags(threshold_enabled: bool = True, variant: str = "sp_f64",
                  minsum_scale: float | None = None, minsum_offset: float | None = None,
                  minsum_self_correct: bool = False) -> int:
    """Flag word of the decode entry points: the reference's threshold switch
    (CFG.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD) and the check-node rule:
    "sp_f64" (the reference, bit-exact), "sp_f32" or "minsum" (build-defined
    binary32 variants; minsum_scale in (0, 1), a multiple of 1/256)."""
    if variant not in N.VARIANTS:
        raise ValueError(f"unknown decoder variant {variant!r}; one of {sorted(N.VARIANTS)}")
    flags = (FLAG_THRESHOLD if threshold_enabled else 0) | N.VARIANTS[variant]
    if minsum_scale is not None:
        if variant != "minsum":
            raise ValueError("minsum_scale applies to variant='minsum' only")
        q = round(minsum_scale * 256)
        if not (1 <= q <= 255) or q != minsum_scale * 256:
            raise ValueError("minsum_scale must be k/256 for k in 1..255")
        flags |= q << N.MINSUM_SCALE_SHIFT
    if minsum_offset is not None:
        if variant != "minsum":
            raise ValueError("minsum_offset applies to variant='minsum' only")
        q = round(minsum_offset * 64)
        if not (0 <= q <= 255) or q != minsum_offset * 64:
            raise ValueError("minsum_offset must be k/64 for k in 0..255")
        flags |= q << N.MINSUM_OFFSET_SHIFT
    if minsum_self_correct:
        if variant != "minsum":
            raise ValueError("minsum_self_correct applies to variant='minsum' only")
        flags |= N.MINSUM_SELF_CORRECT
    return flags


def _ptr(t) -> int | None:
    if t is None:
        return None
    return int(t.data_ptr())


def _stream(stream, device: int) -> int | None:
    """The launch stream: the caller's, else torch's current stream of the code's device
    (not of whatever device happens to be current)."""
    if stream is None:
        return int(torch.cuda.current_stream(device).cuda_stream)
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


def _need_cuda(t, dtype, name, H: "HMatrix | None" = None):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == dtype and t.is_contiguous()):
        raise QkdError(N.ERR_INVALID_ARG, f"{name} must be a contiguous {dtype} CUDA tensor")
    if H is not None and t.device.index != H.device:
        raise QkdError(N.ERR_INVALID_ARG,
                       f"{name} is on {t.device}, the code lives on cuda:{H.device}")


def _frames(t, width: int, name: str, frames: int | None = None) -> int:
    """Frame count of a [F, width] tensor (a 1-D [width] tensor is one frame). The
    kernels read F * width elements, so a ragged or short buffer is an error, never
    a silent floor (the reference's arrays are exactly N or M long)."""
    if t.dim() == 1 and t.numel() == width:
        f = 1
    elif t.dim() == 2 and t.shape[1] == width:
        f = int(t.shape[0])
    else:
        raise QkdError(N.ERR_INVALID_ARG,
                       f"{name} must have shape [F, {width}], got {list(t.shape)}")
    if frames is not None and f != frames:
        raise QkdError(N.ERR_INVALID_ARG, f"{name} holds {f} frames, expected {frames}")
    return f


def _need_vec(t, dtype, count: int, name: str, H: "HMatrix"):
    _need_cuda(t, dtype, name, H)
    if t.numel() != count:
        raise QkdError(N.ERR_INVALID_ARG, f"{name} must hold {count} elements, got {t.numel()}")


class HMatrix:
    """The parity-check matrix (reference H_matrix, array_and_matrix_operations.hpp:16-27),
    uploaded once to one device and immutable afterwards."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)
        info = N.CodeInfo()
        N.check(N.lib().qkd_code_get_info(self._h, C.byref(info)))
        self.num_bit_nodes = info.n_bits
        self.num_check_nodes = info.n_checks
        self.n_edges = info.n_edges
        self.max_bit_nodes_weight = info.max_bit_degree
        self.max_check_nodes_weight = info.max_check_degree
        self.is_regular = bool(info.is_regular)
        self.device = info.device

    # --- constructors (reference readers) ----------------------------------
    @classmethod
    def _make(cls, fn, *args):
        st = C.c_int(0)
        h = fn(*args, C.byref(st))
        if not h:
            raise QkdError(st.value, N.last_error())
        return cls(h)

    @classmethod
    def from_alist(cls, path: str, device: int = 0, sort_rows: bool = False) -> "HMatrix":
        """read_sparse_alist_matrix. sort_rows: accept lines that are not ascending
        by sorting them (QKD_READ_SORT_ROWS) instead of rejecting the file."""
        return cls._make(N.lib().qkd_code_from_alist_ex, str(path).encode(), device,
                         N.READ_SORT_ROWS if sort_rows else 0)

    @classmethod
    def from_dense(cls, path: str, device: int = 0) -> "HMatrix":
        return cls._make(N.lib().qkd_code_from_dense, str(path).encode(), device)

    @classmethod
    def from_check_lists(cls, n_bits: int, check_ptr, check_idx, device: int = 0) -> "HMatrix":
        cp = np.ascontiguousarray(check_ptr, dtype=np.int32)
        ci = np.ascontiguousarray(check_idx, dtype=np.int32)
        return cls._make(N.lib().qkd_code_create, n_bits, cp.size - 1, cp.ctypes.data,
                         ci.ctypes.data, device)

    @classmethod
    def from_dense_array(cls, dense, device: int = 0) -> "HMatrix":
        d = np.asarray(dense)
        ptr, idx = [0], []
        for row in d:
            idx.extend(np.nonzero(row)[0].tolist())
            ptr.append(len(idx))
        return cls.from_check_lists(d.shape[1], ptr, idx, device)

    # --- adjacency ------------------------------------------------------------
    def adjacency(self):
        n, m, e = self.num_bit_nodes, self.num_check_nodes, self.n_edges
        cp = np.zeros(m + 1, np.int32)
        ci = np.zeros(e, np.int32)
        bp = np.zeros(n + 1, np.int32)
        bi = np.zeros(e, np.int32)
        N.check(N.lib().qkd_code_get_adjacency(self._h, cp.ctypes.data, ci.ctypes.data,
                                               bp.ctypes.data, bi.ctypes.data))
        return cp, ci, bp, bi

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            N.lib().qkd_code_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Workspace:
    """Device scratch for one stream (qkd_workspace)."""

    def __init__(self, H: HMatrix):
        st = C.c_int(0)
        h = N.lib().qkd_workspace_create(H.handle, C.byref(st))
        if not h:
            raise QkdError(st.value, N.last_error())
        self._h = C.c_void_p(h)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            N.lib().qkd_workspace_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ws(ws):
    return ws.handle if ws is not None else None


def set_debug_option(name: str, value=None, workspace: "Workspace | None" = None) -> None:
    """qkd_debug_set_option: a debug / A-B option (include/qkd_ldpc.h lists
    them) for `workspace`, or process-wide when None; value None restores the
    default (the product behaviour). The library reads no environment variable."""
    v = None if value is None else str(value).encode()
    N.check(N.lib().qkd_debug_set_option(_ws(workspace), name.encode(), v))


def spec_replays(ws: Workspace, reset: bool = False) -> int:
    """Frames of the QKD path decoded on `ws` whose speculative interval
    iterations could not certify every hard decision and were decoded again
    exactly (qkd_debug_spec_replays); outputs never depend on it."""
    v = C.c_uint64(0)
    N.check(N.lib().qkd_debug_spec_replays(ws.handle, C.byref(v), int(reset)))
    return int(v.value)


def calculate_syndrome(H: HMatrix, bits, stream=None):
    """calculate_syndrome_irregular/_regular: bits [F, N] uint8 -> [F, M] uint8."""
    _need_cuda(bits, torch.uint8, "bits", H)
    f = _frames(bits, H.num_bit_nodes, "bits")
    out = torch.empty((f, H.num_check_nodes), dtype=torch.uint8, device=bits.device)
    N.check(N.lib().qkd_syndrome_batch(H.handle, _ptr(bits), f, _ptr(out), _stream(stream, H.device)))
    return out


@dataclass
class SPResult:
    """SP_result (qkd_ldpc_algorithm.hpp:14-18), one entry per frame."""
    iterations: "torch.Tensor"
    syndromes_match: "torch.Tensor"
    bits: "torch.Tensor | None"


@dataclass
class LDPCResult:
    """LDPC_result (qkd_ldpc_algorithm.hpp:20-24), one entry per frame."""
    iterations: "torch.Tensor"
    syndromes_match: "torch.Tensor"
    keys_match: "torch.Tensor"
    bits: "torch.Tensor | None"


def sum_product_decoding(H: HMatrix, llr, syndrome, max_iterations: int = 50,
                         msg_threshold: float = 100.0, threshold_enabled: bool = True,
                         want_bits: bool = True, workspace=None, stream=None,
                         variant: str = "sp_f64", minsum_scale: float | None = None,
                         minsum_offset: float | None = None, minsum_self_correct: bool = False) -> SPResult:
    """sum_product_decoding_irregular/_regular (qkd_ldpc_algorithm.cpp:3-345), batched.
    llr [F, N] float64, syndrome [F, M] uint8 (0/1)."""
    _need_cuda(llr, torch.float64, "llr", H)
    _need_cuda(syndrome, torch.uint8, "syndrome", H)
    f = _frames(llr, H.num_bit_nodes, "llr")
    _frames(syndrome, H.num_check_nodes, "syndrome", f)
    dev = llr.device
    bits = torch.empty((f, H.num_bit_nodes), dtype=torch.uint8, device=dev) if want_bits else None
    iters = torch.empty(f, dtype=torch.int32, device=dev)
    ok = torch.empty(f, dtype=torch.uint8, device=dev)
    flags = decoder_flags(threshold_enabled, variant, minsum_scale, minsum_offset, minsum_self_correct)
    N.check(N.lib().qkd_decode_batch(H.handle, _ws(workspace), _ptr(llr), _ptr(syndrome), f,
                                     max_iterations, msg_threshold, flags, _ptr(bits), _ptr(iters),
                                     _ptr(ok), _stream(stream, H.device)))
    return SPResult(iters, ok, bits)


# The reference has two twins that differ only in loop bounds; one kernel serves both.
sum_product_decoding_irregular = sum_product_decoding
sum_product_decoding_regular = sum_product_decoding


def qkd_ldpc(H: HMatrix, alice, bob, qber: float, max_iterations: int = 50,
             msg_threshold: float = 100.0, threshold_enabled: bool = True,
             want_bits: bool = False, workspace=None, stream=None,
             variant: str = "sp_f64", minsum_scale: float | None = None,
             minsum_offset: float | None = None, minsum_self_correct: bool = False) -> LDPCResult:
    """QKD_LDPC_irregular/_regular (qkd_ldpc_algorithm.cpp:347-447), batched.
    alice, bob [F, N] uint8 (0/1); one QBER for the batch."""
    _need_cuda(alice, torch.uint8, "alice", H)
    _need_cuda(bob, torch.uint8, "bob", H)
    f = _frames(alice, H.num_bit_nodes, "alice")
    _frames(bob, H.num_bit_nodes, "bob", f)
    dev = alice.device
    bits = torch.empty((f, H.num_bit_nodes), dtype=torch.uint8, device=dev) if want_bits else None
    iters = torch.empty(f, dtype=torch.int32, device=dev)
    ok = torch.empty(f, dtype=torch.uint8, device=dev)
    km = torch.empty(f, dtype=torch.uint8, device=dev)
    flags = decoder_flags(threshold_enabled, variant, minsum_scale, minsum_offset, minsum_self_correct)
    N.check(N.lib().qkd_qkd_ldpc_batch(H.handle, _ws(workspace), _ptr(alice), _ptr(bob), f, qber,
                                       max_iterations, msg_threshold, flags, _ptr(bits),
                                       _ptr(iters), _ptr(ok), _ptr(km), _stream(stream, H.device)))
    return LDPCResult(iters, ok, km, bits)


QKD_LDPC_irregular = qkd_ldpc
QKD_LDPC_regular = qkd_ldpc


def keygen(H: HMatrix, seeds, q_nominal: float, seed_offset: int = 0, workspace=None,
           stream=None):
    """generate_random_bit_array + introduce_errors for frames seeded seeds[k] + seed_offset.
    Returns (alice [F,N] u8, bob [F,N] u8, exact_qber [F] f64) on the device."""
    _need_cuda(seeds, torch.int64, "seeds", H)
    if seeds.dim() != 1:
        raise QkdError(N.ERR_INVALID_ARG, f"seeds must be 1-D, got {list(seeds.shape)}")
    f = seeds.numel()
    dev = seeds.device
    a = torch.empty((f, H.num_bit_nodes), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    q = torch.empty(f, dtype=torch.float64, device=dev)
    N.check(N.lib().qkd_keygen_batch(H.handle, _ws(workspace), _ptr(seeds), seed_offset, f,
                                     q_nominal, _ptr(a), _ptr(b), _ptr(q), _stream(stream, H.device)))
    return a, b, q


@dataclass
class TrialResults:
    iterations: "torch.Tensor"
    syndromes_match: "torch.Tensor"
    keys_match: "torch.Tensor"
    exact_qber: "torch.Tensor"
    counters: "torch.Tensor"      # raw qkd_counters bytes (device)


def run_trials(H: HMatrix, seeds, q_nominal: float, seed_offset: int = 0,
               max_iterations: int = 50, msg_threshold: float = 100.0,
               threshold_enabled: bool = True, workspace=None, stream=None,
               out: TrialResults | None = None, variant: str = "sp_f64",
               minsum_scale: float | None = None, minsum_offset: float | None = None,
               minsum_self_correct: bool = False) -> TrialResults:
    """run_trial (simulation.cpp:161-189) for every frame, fused on the device, plus the
    per-QBER-point counters of simulation.cpp:252-312. seeds: int64 CUDA tensor holding
    the uint64 seed bits."""
    _need_cuda(seeds, torch.int64, "seeds", H)
    if seeds.dim() != 1:
        raise QkdError(N.ERR_INVALID_ARG, f"seeds must be 1-D, got {list(seeds.shape)}")
    f = seeds.numel()
    dev = seeds.device
    if out is not None:
        _need_vec(out.iterations, torch.int32, f, "out.iterations", H)
        _need_vec(out.syndromes_match, torch.uint8, f, "out.syndromes_match", H)
        _need_vec(out.keys_match, torch.uint8, f, "out.keys_match", H)
        _need_vec(out.exact_qber, torch.float64, f, "out.exact_qber", H)
        _need_vec(out.counters, torch.uint8, N.COUNTERS_BYTES, "out.counters", H)
    if out is None:
        out = TrialResults(torch.empty(f, dtype=torch.int32, device=dev),
                           torch.empty(f, dtype=torch.uint8, device=dev),
                           torch.empty(f, dtype=torch.uint8, device=dev),
                           torch.empty(f, dtype=torch.float64, device=dev),
                           torch.empty(N.COUNTERS_BYTES, dtype=torch.uint8, device=dev))
    flags = decoder_flags(threshold_enabled, variant, minsum_scale, minsum_offset, minsum_self_correct)
    N.check(N.lib().qkd_trials_batch(H.handle, _ws(workspace), _ptr(seeds), seed_offset, f,
                                     q_nominal, max_iterations, msg_threshold, flags,
                                     _ptr(out.iterations), _ptr(out.syndromes_match),
                                     _ptr(out.keys_match), _ptr(out.exact_qber),
                                     _ptr(out.counters), _stream(stream, H.device)))
    return out


def interactive_simulation(H: HMatrix, simulation_seed: int, qbers, max_iterations: int = 50,
                           msg_threshold: float = 100.0, threshold_enabled: bool = True,
                           workspace=None, variant: str = "sp_f64") -> dict:
    """QKD_LDPC_interactive_simulation (simulation.cpp:73-137): the QBER points share ONE
    xoshiro256++(simulation_seed) key stream, point after point. Returns host arrays per
    point: exact_qber ("Actual QBER"), errors, iterations, syndromes_match, keys_match,
    success (both flags, "Error reconciliation SUCCESSFUL"). A point whose exact QBER
    would be 0 raises QkdError like the reference's throw; the points before it ran."""
    q = np.ascontiguousarray(qbers, dtype=np.float64)
    p = q.size
    it = np.zeros(p, np.uint32)
    sp = np.zeros(p, np.uint8)
    ko = np.zeros(p, np.uint8)
    ex = np.zeros(p, np.float64)
    er = np.zeros(p, np.uint32)
    done = C.c_size_t(0)
    st = N.lib().qkd_interactive_batch(H.handle, _ws(workspace), simulation_seed, p, q.ctypes.data,
                                       max_iterations, msg_threshold,
                                       decoder_flags(threshold_enabled, variant), it.ctypes.data,
                                       sp.ctypes.data, ko.ctypes.data, ex.ctypes.data, er.ctypes.data,
                                       C.byref(done))
    k = done.value
    out = {"points_done": k, "exact_qber": ex[:k], "errors": er[:k], "iterations": it[:k],
           "syndromes_match": sp[:k].astype(bool), "keys_match": ko[:k].astype(bool),
           "success": (sp[:k] & ko[:k]).astype(bool)}
    if st != N.OK:
        err = QkdError(st, N.last_error())
        err.partial = out
        raise err
    return out


def trace_decode(H: HMatrix, llr, syndrome, max_iterations: int = 50, msg_threshold: float = 100.0,
                 threshold_enabled: bool = True) -> dict:
    """TRACE_SUM_PRODUCT / TRACE_SUM_PRODUCT_LLR of the reference decoder
    (qkd_ldpc_algorithm.cpp:212-330) for one frame, decoded on the device.
    llr [N] float64 and syndrome [M] 0/1 as host arrays. Returns per executed
    iteration t the arrays the reference prints:
      E[t]  check-to-bit messages after the clamp, bit by bit (each bit's checks
            ascending) - the reference's check_to_bit_msg rows
      L[t]  bit totals;  z[t] hard decision;  s[t] its syndrome
      M[t]  bit-to-check messages after the clamp, check by check (each check's
            bits ascending) - bit_to_check_msg; only for iterations that did not
            stop (the reference computes M after the syndrome test)
    and max_llr (MAX_LLR: the largest |E|, |M| over those iterations)."""
    llr = np.ascontiguousarray(llr, dtype=np.float64)
    syn = np.ascontiguousarray(np.asarray(syndrome) != 0, dtype=np.uint8)
    n, m = H.num_bit_nodes, H.num_check_nodes
    cptr, cidx, bptr, bidx = H.adjacency()
    e = len(cidx)
    E = np.zeros((max_iterations, e), np.float64)
    L = np.zeros((max_iterations, n), np.float64)
    it = C.c_uint32()
    ok = C.c_uint8()
    flags = decoder_flags(threshold_enabled, "sp_f64")
    N.check(N.lib().qkd_trace_decode(H.handle, llr.ctypes.data, syn.ctypes.data, max_iterations,
                                     msg_threshold, flags, E.ctypes.data, L.ctypes.data,
                                     C.byref(it), C.byref(ok)))
    t_n = it.value
    E, L = E[:t_n], L[:t_n]
    z = (L <= 0).astype(np.uint8)
    # s: calculate_syndrome of each hard decision
    chk_of = np.repeat(np.arange(m), np.diff(cptr))
    s = np.zeros((t_n, m), np.uint8)
    for t in range(t_n):
        np.bitwise_xor.at(s[t], chk_of, z[t][cidx])
    # M: b2c[j][pos] = clamp(L_i - E[i][k]) for the edge (bit i's k-th check j)
    bit_of_e = np.repeat(np.arange(n), np.diff(bptr))
    pos_in_check = {}
    for j in range(m):
        for p, b in enumerate(cidx[cptr[j]:cptr[j + 1]]):
            pos_in_check[(j, int(b))] = cptr[j] + p
    to_check_order = np.array([pos_in_check[(int(bidx[k]), int(bit_of_e[k]))] for k in range(e)])
    stopped = bool(ok.value)
    t_m = t_n - 1 if stopped else t_n
    M = np.zeros((t_m, e), np.float64)
    max_llr = 0.0
    for t in range(t_m):
        b2c = L[t][bit_of_e] - E[t]
        if threshold_enabled:
            b2c = np.where(b2c > msg_threshold, msg_threshold, np.where(b2c < -msg_threshold, -msg_threshold, b2c))
        M[t][to_check_order] = b2c
        for arr in (E[t], M[t]):
            a = np.abs(arr)
            a = a[~np.isnan(a)]
            if a.size:
                max_llr = max(max_llr, float(a.max()))
    return {"iterations": t_n, "syndromes_match": stopped, "E": E, "L": L, "z": z, "s": s, "M": M,
            "max_llr": max_llr}


def read_counters(counters) -> N.Counters:
    raw = counters.detach().cpu().numpy().tobytes()
    return N.Counters.from_buffer_copy(raw)


def counters_to_stats(c: N.Counters, trials: int, max_iterations: int,
                      initial_qber: float) -> dict:
    """sim_result fields (simulation.hpp:29-43) from exact integer counters. The mean
    and population std match the reference's two-pass double arithmetic to the
    6 significant digits its CSV prints (simulation.cpp:285-312)."""
    sp, ok = int(c.sp_ok), int(c.ldpc_ok)
    mean = std = 0.0
    mn, mx = max_iterations, 0
    if sp > 0:
        s1, s2 = int(c.sum_iters), int(c.sum_iters_sq)
        mean = s1 / sp
        std = ((sp * s2 - s1 * s1) / (sp * sp)) ** 0.5   # exact integer numerator
        mn, mx = int(c.min_iters), int(c.max_iters)
    return {
        "initial_QBER": initial_qber,
        "iterations_successful_sp_mean": mean,
        "iterations_successful_sp_std_dev": std,
        "iterations_successful_sp_min": 0 if mn == max_iterations else mn,
        "iterations_successful_sp_max": mx,
        "ratio_trials_successful_sp": sp / trials,
        "ratio_trials_successful_ldpc": ok / trials,
        "fer": 1.0 - ok / trials,
        "sum_iters_sp": int(c.sum_iters),
    }


def make_seeds(simulation_seed: int, count: int) -> np.ndarray:
    """seeds[k] = k-th raw xoshiro256++(simulation_seed) draw (simulation.cpp:222-228)."""
    out = np.zeros(count, np.uint64)
    N.check(N.lib().qkd_make_seeds(simulation_seed, count, out.ctypes.data))
    return out


def qber_range(begin: float, end: float, step: float) -> list[float]:
    """One row of get_rate_based_QBER_range (simulation.cpp:48-70)."""
    cnt = C.c_size_t(0)
    N.check(N.lib().qkd_qber_range(begin, end, step, None, 0, C.byref(cnt)))
    vals = np.zeros(max(cnt.value, 1), np.float64)
    N.check(N.lib().qkd_qber_range(begin, end, step, vals.ctypes.data, cnt.value, C.byref(cnt)))
    return vals[: cnt.value].tolist()
