"""ctypes binding of the C ABI in include/qkd_ldpc.h (libqkd_ldpc_amd.so).

The library is built in-tree (qkd_ldpc_amd/lib/) by `python -m qkd_ldpc_amd.build`
or __graft_entry__.build(). Loading fails loudly if it is missing: there is
no CPU fallback anywhere in the product path.

torch is imported before the library is loaded so that the process holds one
HIP runtime: torch's bundled libamdhip64 and the system one share the SONAME
libamdhip64.so.7, and the dynamic loader then binds this library to the copy
torch already loaded (device pointers and streams are interchangeable).
"""
from __future__ import annotations

import ctypes as C
import os

try:  # noqa: SIM105 - torch is plumbing (device memory, streams, distributed)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is present in this image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libqkd_ldpc_amd.so")
# A/B experiments only: QKD_AMD_LIB names another build of the same library, and is
# honoured only together with QKD_AMD_DIAGNOSTIC=1 (with a warning on stderr), so
# the product path cannot be swapped silently.
if os.environ.get("QKD_AMD_LIB"):
    if os.environ.get("QKD_AMD_DIAGNOSTIC") == "1":
        import sys as _sys
        LIB_PATH = os.environ["QKD_AMD_LIB"]
        print(f"qkd_ldpc_amd: DIAGNOSTIC build {LIB_PATH} in place of the product library",
              file=_sys.stderr)
    else:
        raise ImportError("QKD_AMD_LIB is set without QKD_AMD_DIAGNOSTIC=1: refusing to load a "
                          "library other than the in-tree product build")

# qkd_status
OK = 0
ERR_INVALID_ARG = 1
ERR_BAD_CODE = 2
ERR_UNSORTED = 3
ERR_QBER_TOO_SMALL = 4
ERR_DEVICE = 5
ERR_OUT_OF_MEMORY = 6
ERR_IO = 7
ERR_UNSUPPORTED = 8

FLAG_THRESHOLD = 0x1
READ_SORT_ROWS = 0x1   # qkd_code_from_alist_ex
# decoder variants (include/qkd_ldpc.h: QKD_VARIANT_*)
VARIANTS = {"sp_f64": 0x00, "sp_f32": 0x10, "minsum": 0x20}
MINSUM_SCALE_SHIFT = 8
MINSUM_OFFSET_SHIFT = 16
MINSUM_SELF_CORRECT = 1 << 24   # QKD_MINSUM_SELF_CORRECT
MINSUM_DEFAULT_SCALE = 0.8125

# Every symbol include/qkd_ldpc.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "qkd_abi_version", "qkd_last_error", "qkd_status_string", "qkd_device_count",
    "qkd_code_create", "qkd_code_from_alist", "qkd_code_from_dense", "qkd_code_destroy",
    "qkd_code_get_info", "qkd_code_get_adjacency", "qkd_workspace_create",
    "qkd_workspace_destroy", "qkd_syndrome_batch", "qkd_decode_batch", "qkd_qkd_ldpc_batch",
    "qkd_keygen_batch", "qkd_trials_batch", "qkd_counters_batch", "qkd_make_seeds",
    "qkd_qber_range", "qkd_debug_phase_cycles", "qkd_debug_spec_replays", "qkd_debug_math", "qkd_debug_phi_sweep", "qkd_trace_decode",
    "qkd_interactive_batch",
    "qkd_code_from_alist_ex", "qkd_debug_decoder_timing", "qkd_debug_bit_order",
    "qkd_counters_merge", "qkd_debug_set_option",
]


class CodeInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_bits", "n_checks", "n_edges", "max_bit_degree",
                                         "max_check_degree", "is_regular", "device")]


class Counters(C.Structure):
    _fields_ = [("frames", C.c_uint64), ("sp_ok", C.c_uint64), ("ldpc_ok", C.c_uint64),
                ("sum_iters", C.c_uint64), ("sum_iters_sq", C.c_uint64),
                ("min_iters", C.c_uint32), ("max_iters", C.c_uint32)]


COUNTERS_BYTES = C.sizeof(Counters)


class QkdError(RuntimeError):
    """A non-OK qkd_status, carrying the library's message (the reference
    raises std::runtime_error for the same conditions)."""

    def __init__(self, status: int, message: str):
        super().__init__(message or f"qkd status {status}")
        self.status = status


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -m qkd_ldpc_amd.build` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        P, I32, U32, U64, SZ, D = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64, C.c_size_t, C.c_double
        st = C.c_int
        sig = {
            "qkd_abi_version": (C.c_int, []),
            "qkd_last_error": (C.c_char_p, []),
            "qkd_status_string": (C.c_char_p, [st]),
            "qkd_device_count": (C.c_int, []),
            "qkd_code_create": (P, [I32, I32, P, P, C.c_int, C.POINTER(st)]),
            "qkd_code_from_alist": (P, [C.c_char_p, C.c_int, C.POINTER(st)]),
            "qkd_code_from_alist_ex": (P, [C.c_char_p, C.c_int, U32, C.POINTER(st)]),
            "qkd_code_from_dense": (P, [C.c_char_p, C.c_int, C.POINTER(st)]),
            "qkd_code_destroy": (None, [P]),
            "qkd_code_get_info": (st, [P, C.POINTER(CodeInfo)]),
            "qkd_code_get_adjacency": (st, [P, P, P, P, P]),
            "qkd_workspace_create": (P, [P, C.POINTER(st)]),
            "qkd_workspace_destroy": (None, [P]),
            "qkd_syndrome_batch": (st, [P, P, SZ, P, P]),
            "qkd_decode_batch": (st, [P, P, P, P, SZ, U32, D, U32, P, P, P, P]),
            "qkd_qkd_ldpc_batch": (st, [P, P, P, P, SZ, D, U32, D, U32, P, P, P, P, P]),
            "qkd_keygen_batch": (st, [P, P, P, U64, SZ, D, P, P, P, P]),
            "qkd_trials_batch": (st, [P, P, P, U64, SZ, D, U32, D, U32, P, P, P, P, P, P]),
            "qkd_counters_batch": (st, [P, P, P, SZ, P, C.c_int, P]),
            "qkd_counters_merge": (st, [P, SZ, P, C.c_int, P]),
            "qkd_make_seeds": (st, [U64, SZ, P]),
            "qkd_qber_range": (st, [D, D, D, P, SZ, C.POINTER(SZ)]),
            "qkd_debug_phase_cycles": (st, [P, P]),
            "qkd_debug_decoder_timing": (st, [P, C.c_int, C.POINTER(D), C.POINTER(U64)]),
            "qkd_debug_spec_replays": (st, [P, P, C.c_int]),
            "qkd_debug_math": (st, [C.c_int, P, P, SZ, P]),
            "qkd_debug_phi_sweep": (st, [C.c_int, C.c_uint32, C.c_uint32, P]),
            "qkd_debug_bit_order": (st, [I32, I32, P, P, C.c_char_p, P, P, C.POINTER(I32)]),
            "qkd_debug_set_option": (st, [P, C.c_char_p, C.c_char_p]),
            "qkd_interactive_batch": (st, [P, P, C.c_uint64, SZ, P, C.c_uint32, C.c_double, C.c_uint32,
                                           P, P, P, P, P, P]),
            "qkd_trace_decode": (st, [P, P, P, U32, D, U32, P, P, P, P]),
        }
        diagnostic = os.environ.get("QKD_AMD_LIB") and os.environ.get("QKD_AMD_DIAGNOSTIC") == "1"
        for name, (res, args) in sig.items():
            if diagnostic and not hasattr(L, name):
                continue          # an older build in an A/B run may lack newer debug entries
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return lib().qkd_last_error().decode(errors="replace")


def check(status: int) -> None:
    if status != OK:
        raise QkdError(status, last_error())
