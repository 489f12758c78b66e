"""ctypes binding for the oracle (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker. The product (qkd_ldpc_amd/) never
imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
        f64p = np.ctypeslib.ndpointer(np.float64, flags="C")
        u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
        L.orc_code_from_alist.restype = P
        L.orc_code_from_alist.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.orc_code_from_dense.restype = P
        L.orc_code_from_dense.argtypes = [u8p, C.c_int, C.c_int]
        L.orc_code_from_lists.restype = P
        L.orc_code_from_lists.argtypes = [C.c_int, C.c_int, i32p, i32p, i32p, i32p, C.c_int, C.c_int]
        L.orc_code_free.argtypes = [P]
        L.orc_code_dims.argtypes = [P, i32p]
        L.orc_code_lists.argtypes = [P, i32p, i32p, i32p, i32p]
        L.orc_seeds.argtypes = [C.c_uint64, C.c_size_t, u64p]
        L.orc_libm_array.argtypes = [C.c_int, f64p, f64p, C.c_size_t]
        L.orc_keygen.restype = C.c_double
        L.orc_keygen.argtypes = [C.c_uint64, C.c_int, C.c_double, i32p, i32p]
        L.orc_syndrome.argtypes = [P, i32p, i32p]
        L.orc_decode.restype = C.c_int
        L.orc_decode.argtypes = [P, f64p, i32p, C.c_int, C.c_double, C.c_int, i32p,
                                 C.POINTER(C.c_int), C.POINTER(C.c_int), P, C.POINTER(C.c_int), P,
                                 C.POINTER(C.c_double), P]
        L.orc_qkd_ldpc.argtypes = [P, i32p, i32p, C.c_double, C.c_int, C.c_double, C.c_int,
                                   C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), P]
        L.orc_run_trial.restype = C.c_int
        L.orc_run_trial.argtypes = [P, C.c_double, C.c_uint64, C.c_int, C.c_double, C.c_int,
                                    C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(C.c_double)]
        L.orc_trials.restype = C.c_int
        L.orc_trials.argtypes = [P, C.c_double, u64p, C.c_uint64, C.c_size_t, C.c_int, C.c_double,
                                 C.c_int, C.c_int, i32p, i32p, i32p, f64p]
        L.orc_interactive.restype = C.c_int
        L.orc_interactive.argtypes = [P, C.c_uint64, f64p, C.c_int, C.c_int, C.c_double, C.c_int,
                                      i32p, i32p, i32p, f64p, i32p]
        _lib = L
    return _lib


class Code:
    """The reference's H_matrix as the oracle holds it (jagged, file order)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("oracle: failed to build code")
        self.h = handle
        d = np.zeros(6, np.int32)
        lib().orc_code_dims(self.h, d)
        self.n, self.m, self.e, self.max_dv, self.max_dc, self.is_regular = (int(x) for x in d)

    @classmethod
    def from_alist(cls, path: str) -> "Code":
        err = C.create_string_buffer(512)
        h = lib().orc_code_from_alist(path.encode(), err, 512)
        if not h:
            raise RuntimeError(err.value.decode())
        return cls(h)

    @classmethod
    def from_dense(cls, dense: np.ndarray) -> "Code":
        d = np.ascontiguousarray(dense, dtype=np.uint8)
        return cls(lib().orc_code_from_dense(d, d.shape[0], d.shape[1]))

    @classmethod
    def from_lists(cls, z) -> "Code":
        """From a mapping holding bit_off/bit_idx/chk_off/chk_idx/dims (the golden npz)."""
        bo = np.ascontiguousarray(z["bit_off"], np.int32)
        bi = np.ascontiguousarray(z["bit_idx"], np.int32)
        co = np.ascontiguousarray(z["chk_off"], np.int32)
        ci = np.ascontiguousarray(z["chk_idx"], np.int32)
        d = np.asarray(z["dims"])
        return cls(lib().orc_code_from_lists(int(d[0]), int(d[1]), bo, bi, co, ci, int(d[2]),
                                             int(d[3])))

    def lists(self):
        bo = np.zeros(self.n + 1, np.int32)
        co = np.zeros(self.m + 1, np.int32)
        bi = np.zeros(self.e, np.int32)
        ci = np.zeros(self.e, np.int32)
        lib().orc_code_lists(self.h, bo, bi, co, ci)
        return bo, bi, co, ci

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_code_free(self.h)
            self.h = None

    # --- reference functions -------------------------------------------------
    def syndrome(self, bits) -> np.ndarray:
        b = np.ascontiguousarray(bits, dtype=np.int32)
        out = np.zeros(self.m, np.int32)
        lib().orc_syndrome(self.h, b, out)
        return out

    def decode(self, llr, syndrome, max_it=50, thr=100.0, thr_enable=True,
               fingerprints=False, ltrace=False, etrace=False):
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        syn = np.ascontiguousarray(syndrome, dtype=np.int32)
        out = np.zeros(self.n, np.int32)
        it, ok, nfp, mx = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        fp = np.zeros(2 * max_it, np.uint64) if fingerprints else None
        lt = np.zeros((max_it, self.n), np.float64) if ltrace else None
        et = np.zeros((max_it, self.e), np.float64) if etrace else None
        lib().orc_decode(self.h, llr, syn, max_it, thr, int(thr_enable), out, C.byref(it),
                         C.byref(ok), fp.ctypes.data if fp is not None else None, C.byref(nfp),
                         lt.ctypes.data if lt is not None else None, C.byref(mx),
                         et.ctypes.data if et is not None else None)
        res = {"iters": it.value, "sp_ok": bool(ok.value), "out": out, "max_llr": mx.value}
        if fp is not None:
            res["fingerprints"] = [int(x) for x in fp[: nfp.value]]
        if lt is not None:
            res["ltrace"] = lt[: it.value]
        if et is not None:
            res["etrace"] = et[: it.value]     # c2b after the clamp, bit-major (bit_off order)
        return res

    def qkd_ldpc(self, alice, bob, q, max_it=50, thr=100.0, thr_enable=True):
        a = np.ascontiguousarray(alice, dtype=np.int32)
        b = np.ascontiguousarray(bob, dtype=np.int32)
        it, sp, ko = C.c_int(), C.c_int(), C.c_int()
        out = np.zeros(self.n, np.int32)
        lib().orc_qkd_ldpc(self.h, a, b, q, max_it, thr, int(thr_enable), C.byref(it), C.byref(sp),
                           C.byref(ko), out.ctypes.data)
        return {"iters": it.value, "sp_ok": bool(sp.value), "key_ok": bool(ko.value), "out": out}

    def run_trial(self, q_nom, seed, max_it=50, thr=100.0, thr_enable=True):
        it, sp, ko, q = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        rc = lib().orc_run_trial(self.h, q_nom, seed, max_it, thr, int(thr_enable), C.byref(it),
                                 C.byref(sp), C.byref(ko), C.byref(q))
        if rc != 0:
            raise RuntimeError(f"Key size '{self.n}' is too small for QBER.")
        return {"iters": it.value, "sp_ok": bool(sp.value), "key_ok": bool(ko.value),
                "exact_q": q.value}

    def trials(self, q_nom, seeds, offset=0, max_it=50, thr=100.0, thr_enable=True, threads=None):
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        f = seeds.size
        it = np.zeros(f, np.int32)
        sp = np.zeros(f, np.int32)
        ko = np.zeros(f, np.int32)
        q = np.zeros(f, np.float64)
        threads = threads or os.cpu_count() or 1
        rc = lib().orc_trials(self.h, q_nom, seeds, offset, f, max_it, thr, int(thr_enable),
                              threads, it, sp, ko, q)
        if rc != 0:
            raise RuntimeError(f"Key size '{self.n}' is too small for QBER.")
        return {"iters": it, "sp_ok": sp.astype(bool), "key_ok": ko.astype(bool), "exact_q": q}


def interactive(code: "Code", sim_seed: int, q_nom, max_it=50, thr=100.0, thr_enable=True):
    """QKD_LDPC_interactive_simulation (simulation.cpp:73-137) over the points q_nom:
    one shared xoshiro256++ stream. Returns per-point arrays and `stop`, the index
    of the point whose exact QBER was 0 (the reference throws there) or -1."""
    q = np.ascontiguousarray(q_nom, dtype=np.float64)
    p = q.size
    it = np.zeros(p, np.int32)
    sp = np.zeros(p, np.int32)
    ko = np.zeros(p, np.int32)
    ex = np.zeros(p, np.float64)
    er = np.zeros(p, np.int32)
    stop = lib().orc_interactive(code.h, sim_seed, q, p, max_it, thr, int(thr_enable), it, sp, ko, ex, er)
    return {"iters": it, "sp_ok": sp.astype(bool), "key_ok": ko.astype(bool), "exact_q": ex,
            "errors": er, "stop": int(stop)}


def libm(which: str, x) -> np.ndarray:
    """glibc tanh ('tanh') or atanh ('atanh') of every element."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    lib().orc_libm_array(0 if which == "tanh" else 1, x, y, x.size)
    return y


def seeds(sim_seed: int, count: int) -> np.ndarray:
    out = np.zeros(count, np.uint64)
    lib().orc_seeds(sim_seed, count, out)
    return out


def keygen(seed: int, n: int, q_nom: float):
    a = np.zeros(n, np.int32)
    b = np.zeros(n, np.int32)
    q = lib().orc_keygen(seed, n, q_nom, a, b)
    return a, b, q


def batch_stats(iters, sp_ok, key_ok, exact_q, trials, max_it):
    """Per-QBER-point reduction of QKD_LDPC_batch_simulation (simulation.cpp:252-312)."""
    iters = np.asarray(iters)
    sp = np.asarray(sp_ok, bool)
    ko = np.asarray(key_ok, bool)
    n_sp = int(sp.sum())
    n_ldpc = int((sp & ko).sum())
    mx, mn, mean, std = 0, max_it, 0.0, 0.0
    if n_sp > 0:
        its = iters[sp]
        mx = int(its.max())
        mn = int(its.min())
        for v in its:                        # serial double sum, trial order
            mean += float(v)
        mean /= float(n_sp)
        acc = 0.0
        for v in its:
            acc += (float(v) - mean) ** 2
        std = (acc / float(n_sp)) ** 0.5
    return {
        "initial_QBER": float(exact_q[0]),
        "iterations_successful_sp_mean": mean,
        "iterations_successful_sp_std_dev": std,
        "iterations_successful_sp_min": 0 if mn == max_it else mn,
        "iterations_successful_sp_max": mx,
        "ratio_trials_successful_sp": n_sp / trials,
        "ratio_trials_successful_ldpc": n_ldpc / trials,
        "fer": 1.0 - n_ldpc / trials,
        "sum_iters_sp": int(iters[sp].sum()) if n_sp else 0,
    }
