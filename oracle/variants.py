"""Models of the build-defined decoder variants (QKD_VARIANT_MINSUM).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the min-sum
kernel. The reference has no min-sum decoder (SURVEY.md §8(d), config 5:
"build-defined, not in the reference"); this is the specification of the one in
include/qkd_ldpc.h, written with numpy binary32 arithmetic so that every
operation rounds exactly as the kernel's does:

  schedule      the reference's flooding loop (qkd_ldpc_algorithm.cpp:212-330)
  b2c           LLR_i at iteration 0 (:188), else clamp(total_i - c2b) (:303-316)
  c2b           (-1)^(s_j + #negative other b2c) * max(scale * min over the other
                |b2c| - offset, 0) (offset 0: plain normalised min-sum; NaN inputs
                ignored by the min, as fminf, which is +inf when no other edge
                has a number), then clamp (:246-249)
  self-correct  (QKD_MINSUM_SELF_CORRECT, Savin's self-corrected min-sum) from the
                second iteration on, a b2c whose sign differs from the edge's
                previous b2c, both nonzero, is erased to 0 before the check rule
  total         float(LLR_i) + c2b_0 + c2b_1 + ... in ascending check order (:256-267)
  stop          H z == s, z_i = total_i <= 0 (:277-285)
"""
from __future__ import annotations

import numpy as np


class MinSumModel:
    def __init__(self, n: int, m: int, check_ptr, check_idx):
        co = np.asarray(check_ptr, np.int64)
        ci = np.asarray(check_idx, np.int64)
        self.n, self.m = n, m
        e = len(ci)
        deg = np.diff(co)
        self.dc = int(deg.max())
        # check-side slots: edge ids in check order, -1 pad
        self.cslot = np.full((m, self.dc), -1, np.int64)
        for k in range(self.dc):
            has = deg > k
            self.cslot[has, k] = co[:-1][has] + k
        self.bit_of_edge = ci
        self.chk_of_edge = np.repeat(np.arange(m), deg)
        # bit-side slots: edge ids in ascending check order per bit
        order = np.lexsort((self.chk_of_edge, ci))            # by bit, then check
        bdeg = np.bincount(ci, minlength=n)
        self.dv = int(bdeg.max())
        bptr = np.concatenate([[0], np.cumsum(bdeg)])
        self.bslot = np.full((n, self.dv), -1, np.int64)
        for k in range(self.dv):
            has = bdeg > k
            self.bslot[has, k] = order[bptr[:-1][has] + k]
        self.e = e

    def syndrome(self, bits):
        """bits [F, N] 0/1 -> [F, M] 0/1 (calculate_syndrome)."""
        b = np.asarray(bits, np.uint8)
        pad = np.concatenate([b, np.zeros((b.shape[0], 1), np.uint8)], axis=1)
        idx = np.where(self.cslot >= 0, self.bit_of_edge[np.maximum(self.cslot, 0)], self.n)
        return np.bitwise_xor.reduce(pad[:, idx], axis=2)

    @staticmethod
    def _clamp(v, thr):
        return np.where(v > thr, thr, np.where(v < -thr, -thr, v)).astype(np.float32)

    def decode(self, llr, syndrome, max_it=50, thr=100.0, thr_enable=True, scale=0.8125, offset=0.0,
               self_correct=False):
        """llr [F, N] float64, syndrome [F, M] -> (bits [F, N] u8, iterations [F], sp_ok [F])."""
        llr32 = np.asarray(llr, np.float64).astype(np.float32)
        syn = np.asarray(syndrome, np.uint8)
        F = llr32.shape[0]
        thr32 = np.float32(thr)
        sc = np.float32(scale)
        c2b = np.zeros((F, self.e), np.float32)
        total = llr32.copy()
        out_bits = np.zeros((F, self.n), np.uint8)
        iters = np.full(F, max_it, np.int64)
        ok = np.zeros(F, np.uint8)
        live = np.ones(F, bool)
        valid = self.cslot >= 0
        cs = np.maximum(self.cslot, 0)
        prev = None
        for it in range(max_it):
            b2c = total[:, self.bit_of_edge]
            if it > 0:
                b2c = (b2c - c2b).astype(np.float32)
                if thr_enable:
                    b2c = self._clamp(b2c, thr32)
                if self_correct:
                    with np.errstate(invalid="ignore"):
                        er = (prev != 0) & (b2c != 0) & ((b2c < 0) != (prev < 0))
                    b2c = np.where(er, np.float32(0), b2c).astype(np.float32)
            prev = b2c
            B = b2c[:, cs]                                           # [F, M, DC]
            mag = np.where(valid[None], np.abs(B), np.float32(np.inf)).astype(np.float32)
            negb = ((B < 0) & valid[None]).astype(np.uint8)
            neg_all = syn ^ np.bitwise_xor.reduce(negb, axis=2)      # [F, M]
            new = np.zeros_like(c2b)
            for k in range(self.dc):
                others = np.delete(mag, k, axis=2)
                # (NaN magnitudes ignored, as fminf; +inf when no other edge has a number)
                mn = np.fmin.reduce(others, axis=2, initial=np.inf) if others.shape[2] else np.full(mag.shape[:2], np.inf, np.float32)
                mn = mn.astype(np.float32)
                v = (sc * mn).astype(np.float32)
                if offset > 0:
                    v = np.fmax((v - np.float32(offset)).astype(np.float32), np.float32(0))
                neg = neg_all ^ negb[:, :, k]
                v = np.where(neg == 1, -v, v).astype(np.float32)
                if thr_enable:
                    v = self._clamp(v, thr32)
                col = valid[:, k]
                new[:, self.cslot[col, k]] = v[:, col]
            c2b = new
            acc = llr32.copy()
            for k in range(self.dv):
                has = self.bslot[:, k] >= 0
                add = c2b[:, np.maximum(self.bslot[:, k], 0)]
                acc = np.where(has[None], (acc + add).astype(np.float32), acc)
            total = acc
            z = (total <= 0).astype(np.uint8)
            match = (self.syndrome(z) == syn).all(axis=1)
            fin = live & match
            out_bits[fin] = z[fin]
            iters[fin] = it + 1
            ok[fin] = 1
            live &= ~match
            if not live.any():
                break
        out_bits[live] = (total[live] <= 0).astype(np.uint8)
        return out_bits, iters, ok


def _psi_np(x):
    """Signed psi(|x|) = sign(x) phi(|x|) / ln 2 in numpy (|x| limited to [1e-30, 80]):
    the statistical stand-in for the device's evaluation (qkd_debug_math which = 2)."""
    a = np.abs(np.asarray(x, np.float32)).astype(np.float64)
    a = np.where(a < 1e-30, 1e-30, np.where(a > 80.0, 80.0, a))
    p = np.log1p(2 * np.exp(-a) / -np.expm1(-a)) / np.log(2.0)
    return np.where(np.asarray(x) < 0, -p, p).astype(np.float32)


def _phi_out_np(s):
    """phi(S ln 2) of a psi-unit sum S (limited to 115): stand-in for which = 3."""
    S = np.minimum(np.asarray(s, np.float64), 115.0) * np.log(2.0)
    with np.errstate(divide="ignore"):
        return np.log1p(2 * np.exp(-S) / -np.expm1(-S)).astype(np.float32)


def sp_f32_decode(model: MinSumModel, llr, syndrome, max_it=50, thr=100.0, thr_enable=True,
                  trace=None, tanh_half=None, two_atanh=None, trace_ref=None):
    """Model of QKD_VARIANT_SP_F32 -> (bits, iterations, sp_ok): binary32 messages and
    totals, the check rule in Gallager's form (qkd_decode.h RuleMath<kRuleSp32>):
      p_k  = sign(b2c_k) psi(|b2c_k|)                       (published per edge)
      S    = sum over the other edges of |p_m|, ascending    (binary32 adds)
      c2b  = (-1)^(s_j + #negative other p) phi(S ln 2), clamped
    With the device's own elementwise steps plugged in (tanh_half = the published
    value, qkd_debug_math which = 2; two_atanh = phi(S ln 2), which = 3) it is the
    kernel's specification bit for bit; with the numpy stand-ins (the default) it
    tracks the kernel statistically.
    trace: optional list; per iteration it receives (n_nan_messages, n_zero_b2c, n_errors
    of the hard decision vs trace_ref if given)."""
    llr32 = np.asarray(llr, np.float64).astype(np.float32)
    syn = np.asarray(syndrome, np.uint8)
    F = llr32.shape[0]
    thr32 = np.float32(thr)
    c2b = np.zeros((F, model.e), np.float32)
    total = llr32.copy()
    iters = np.full(F, max_it, np.int64)
    ok = np.zeros(F, np.uint8)
    out_bits = np.zeros((F, model.n), np.uint8)
    live = np.ones(F, bool)
    valid = model.cslot >= 0
    cs = np.maximum(model.cslot, 0)
    with np.errstate(all="ignore"):
        for it in range(max_it):
            b2c = total[:, model.bit_of_edge]
            if it > 0:
                b2c = (b2c - c2b).astype(np.float32)
                if thr_enable:
                    b2c = MinSumModel._clamp(b2c, thr32)
            pub = (tanh_half(b2c) if tanh_half else _psi_np(b2c)).astype(np.float32)
            P = pub[:, cs]
            new = np.zeros_like(c2b)
            for k in range(model.dc):
                # extrinsic psi sum over the other edges, ascending, and their sign parity
                S = np.zeros(P.shape[:2], np.float32)
                neg = syn.astype(np.uint8).copy()
                for j in range(model.dc):
                    if j != k:
                        on = valid[None, :, j]
                        S = np.where(on, (S + np.abs(P[:, :, j])).astype(np.float32), S)
                        neg = np.where(on, neg ^ (P[:, :, j] < 0).astype(np.uint8), neg)
                v = (two_atanh(S) if two_atanh else _phi_out_np(S)).astype(np.float32)
                v = np.where(neg == 1, -v, v).astype(np.float32)
                if thr_enable:
                    v = MinSumModel._clamp(v, thr32)
                col = valid[:, k]
                new[:, model.cslot[col, k]] = v[:, col]
            if trace is not None:
                trace.append((int(np.isnan(new).sum()), int((b2c == 0).sum())))
            c2b = new
            acc = llr32.copy()
            for k in range(model.dv):
                has = model.bslot[:, k] >= 0
                add = c2b[:, np.maximum(model.bslot[:, k], 0)]
                acc = np.where(has[None], (acc + add).astype(np.float32), acc)
            total = acc
            z = (total <= 0).astype(np.uint8)
            if trace is not None and trace_ref is not None:
                trace[-1] = trace[-1] + (int((z != trace_ref).sum()),)
            match = (model.syndrome(z) == syn).all(axis=1)
            fin = live & match
            out_bits[fin] = z[fin]
            iters[fin] = it + 1
            ok[fin] = 1
            live &= ~match
            if not live.any():
                break
        out_bits[live] = (total[live] <= 0).astype(np.uint8)
    return out_bits, iters, ok
