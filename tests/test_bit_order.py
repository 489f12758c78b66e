"""The split decoder's internal bit order (host.cpp internal_bit_order), on CPU
through qkd_debug_bit_order: a permutation of the bits; each task's last-row
edges on consecutive internal bits (the global slots a check phase touches come
in runs); the LDS bank pass keeps those runs and cuts the check
phase's modelled bank excess (tools/bank_model.py's measure) well below both the
code's original order and the unbalanced runs."""
import ctypes as C
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN


@pytest.fixture(scope="module")
def code():
    z = np.load(os.path.join(GOLDEN, "code_n10240.npz"))
    return int(z["dims"][0]), int(z["dims"][1]), np.ascontiguousarray(z["chk_off"], np.int32), \
        np.ascontiguousarray(z["chk_idx"], np.int32)


def bit_order(code, mode):
    from qkd_ldpc_amd import _native as N
    n, m, cp, ci = code
    nt = C.c_int32(0)
    N.check(N.lib().qkd_debug_bit_order(n, m, cp.ctypes.data, ci.ctypes.data, None, None, None, C.byref(nt)))
    perm = np.zeros(n, np.int32)
    plan = np.zeros(nt.value * 64, np.uint32)
    N.check(N.lib().qkd_debug_bit_order(n, m, cp.ctypes.data, ci.ctypes.data,
                                        mode.encode() if mode else None, perm.ctypes.data, plan.ctypes.data,
                                        C.byref(nt)))
    return perm, plan.reshape(nt.value, 64)


def bank_excess(n, plan, inv, bdeg, n_pad):
    """Summed over tasks and half-waves: the busiest bank pair's count - 1 among the
    distinct not-last-row slots x = row * n_pad + internal bit (x mod 32)."""
    ex = 0
    for task in plan:
        for h in (task[:32], task[32:]):
            xs = set()
            for w in h:
                b, r = int(w & 0xFFFFFF), int(w >> 24)
                if b < n and r != bdeg[b] - 1:
                    xs.add(r * n_pad + int(inv[b]))
            if xs:
                ex += np.bincount(np.array(sorted(xs)) % 32, minlength=32).max() - 1
    return ex


def test_internal_order_runs_and_banks(code):
    n, m, cp, ci = code
    bdeg = np.bincount(ci, minlength=n)
    n_pad = (n + 1 + 63) // 64 * 64
    out = {}
    for mode in (None, "runs", "identity"):
        perm, plan = bit_order(code, mode)
        assert sorted(perm.tolist()) == list(range(n)), mode
        inv = np.empty(n, np.int64)
        inv[perm] = np.arange(n)
        if mode != "identity":
            # every task's last-row bits occupy one run of consecutive internal bits
            for task in plan:
                q = sorted(int(inv[w & 0xFFFFFF]) for w in task
                           if (w & 0xFFFFFF) < n and (w >> 24) == bdeg[w & 0xFFFFFF] - 1)
                assert not q or q[-1] - q[0] == len(q) - 1
        out[mode] = bank_excess(n, plan, inv, bdeg, n_pad) / len(plan)
    # runs alone cost a little over the original order; the bank pass more than halves it
    assert out[None] < 0.5 * min(out["runs"], out["identity"]), out


def test_bit_order_is_deterministic(code):
    a, _ = bit_order(code, None)
    b, _ = bit_order(code, None)
    assert (a == b).all()
