"""Models of the build-defined decoder variants (QKD_VARIANT_MINSUM).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the min-sum
kernel. The reference has no min-sum decoder (SURVEY.md §8(d), config 5:
"build-defined, not in the reference"); this is the specification of the one in
include/qkd_ldpc.h, written with numpy binary32 arithmetic so that every
operation rounds exactly as the kernel's does:

  schedule      the reference's flooding loop (qkd_ldpc_algorithm.cpp:212-330)
  b2c           LLR_i at iteration 0 (:188), else clamp(total_i - c2b) (:303-316)
  c2b           scale * (-1)^(s_j + #negative other b2c) * min over the other |b2c|
                (NaN inputs ignored by the min, as fminf), then clamp (:246-249)
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

    def decode(self, llr, syndrome, max_it=50, thr=100.0, thr_enable=True, scale=0.8125):
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
        for it in range(max_it):
            b2c = total[:, self.bit_of_edge]
            if it > 0:
                b2c = (b2c - c2b).astype(np.float32)
                if thr_enable:
                    b2c = self._clamp(b2c, thr32)
            B = b2c[:, cs]                                           # [F, M, DC]
            mag = np.where(valid[None], np.abs(B), np.float32(np.inf)).astype(np.float32)
            negb = ((B < 0) & valid[None]).astype(np.uint8)
            neg_all = syn ^ np.bitwise_xor.reduce(negb, axis=2)      # [F, M]
            new = np.zeros_like(c2b)
            for k in range(self.dc):
                others = np.delete(mag, k, axis=2)
                mn = np.fmin.reduce(others, axis=2) if others.shape[2] else np.full(mag.shape[:2], np.inf, np.float32)
                mn = mn.astype(np.float32)
                v = (sc * mn).astype(np.float32)
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


def sp_f32_decode(model: MinSumModel, llr, syndrome, max_it=50, thr=100.0, thr_enable=True,
                  trace=None, tanh_half=None, two_atanh=None, trace_ref=None):
    """Model of QKD_VARIANT_SP_F32 -> (bits, iterations, sp_ok). With the device's own
    elementwise tanh(x/2) / 2 atanh(x) plugged in (qkd_debug_math which = 2 / 3) it is
    the kernel's specification bit for bit; with numpy's float32 tanh / arctanh
    (the default) it tracks the kernel statistically.
    trace: optional list; per iteration it receives (n_nan_messages, n_zero_b2c, n_errors
    of the hard decision vs trace_ref if given). tanh_half / two_atanh: optional
    replacements of the two transcendental steps (e.g. the device's, through
    qkd_debug_math) taking and returning float32 arrays."""
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
            t = (tanh_half(b2c) if tanh_half else np.tanh(b2c * np.float32(0.5))).astype(np.float32)
            T = t[:, cs]
            sgn = np.where(syn == 1, np.float32(-1), np.float32(1)).astype(np.float32)
            new = np.zeros_like(c2b)
            for k in range(model.dc):
                # extrinsic product over the other edges, ascending, no division
                r = sgn.copy()
                for j in range(model.dc):
                    if j != k:
                        r = np.where(valid[None, :, j], (r * T[:, :, j]).astype(np.float32), r)
                if two_atanh:
                    v = two_atanh(r).astype(np.float32)
                else:
                    kmax = np.float32(np.nextafter(np.float32(1), np.float32(0)))
                    r = np.where(r > kmax, kmax, np.where(r < -kmax, -kmax, r))
                    v = (np.float32(2) * np.arctanh(r)).astype(np.float32)
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
