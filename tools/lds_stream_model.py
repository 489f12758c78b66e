"""LDS bank model of the split decoder's check-phase access streams (CPU; the
banking rules of MI355X_MICROARCH.md §LDS): per task and wave-instruction, the
extra LDS cycles (distinct addresses on the busiest bank of each lane group,
minus one) of
  * the slot read (ds_read_b64: 2 groups of 32 lanes, bank = dword mod 64) and
    slot write (ds_write_b64: 4 groups of 16 lanes, dword mod 32), lanes of
    global slots excluded (their LDS addresses are out of range: no banking,
    tools/mb/lds_bank_mb.hip read_oob_only);
  * the extrinsic-sum row reads row[start + k], k < 6, as the compiler emits
    them (3 x ds_read2_b64: each access 4 groups of 16 lanes, dword mod 32);
  * the segment-weight reads (ds_read2_b64 + ds_read_b64 of the wtab row).
Layout: SplitLds of the config-2 speculative launch (tools/mb/gen_lds_stream.py).

    python tools/lds_stream_model.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "mb"))


def group_extra(addrs, nbank, width=2):
    """Extra cycles of one lane group: addrs = byte addresses (in-range lanes only)
    of `width`-dword accesses; identical addresses broadcast."""
    if len(addrs) == 0:
        return 0
    ua = np.unique(addrs)
    banks = np.concatenate([(ua // 4 + w) % nbank for w in range(width)])
    return int(np.bincount(banks, minlength=nbank).max()) - 1


def plan_tasks():
    """Per task and lane: (original bit, row, check, segment start, degree)."""
    from qkd_ldpc_amd import _native as N
    g = np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))
    n, m = int(g["dims"][0]), int(g["dims"][1])
    cptr = np.ascontiguousarray(g["chk_off"], np.int32)
    cidx = np.ascontiguousarray(g["chk_idx"], np.int32)
    L = N.lib()
    nt = C.c_int32(0)
    N.check(L.qkd_debug_bit_order(n, m, cptr.ctypes.data, cidx.ctypes.data, None, None, None, C.byref(nt)))
    perm = np.zeros(n, np.int32)
    plan = np.zeros(nt.value * 64, np.uint32)
    N.check(L.qkd_debug_bit_order(n, m, cptr.ctypes.data, cidx.ctypes.data, None, perm.ctypes.data,
                                  plan.ctypes.data, C.byref(nt)))
    # the r-th check (ascending) of each bit
    bchk = [[] for _ in range(n)]
    for j in range(m):
        for k in range(cptr[j], cptr[j + 1]):
            bchk[cidx[k]].append(j)
    b = (plan & 0xFFFFFF).astype(np.int64)
    r = (plan >> 24).astype(np.int64)
    chk = np.array([bchk[bb][rr] if bb < n else -1 - i for i, (bb, rr) in enumerate(zip(b, r))], np.int64)
    chk = chk.reshape(-1, 64)
    start = np.zeros_like(chk)
    deg = np.zeros_like(chk)
    for t in range(chk.shape[0]):
        l = 0
        while l < 64:
            e = l
            while e + 1 < 64 and chk[t, e + 1] == chk[t, l]:
                e += 1
            if chk[t, l] < 0:       # idle lane: plan_seg(0, lane, 1), a degree-1 segment of its own
                start[t, l], deg[t, l] = l, 1
            else:
                start[t, l:e + 1] = l
                deg[t, l:e + 1] = e - l + 1
            l = e + 1
    return n, m, nt.value, perm, b.reshape(-1, 64), r.reshape(-1, 64), chk, start, deg


def main():
    from gen_lds_stream import split_lds
    n, m, nt, perm, b, r, chk, start, deg = plan_tasks()
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    n_pad = (n + 1 + 63) // 64 * 64
    DC, NW = 6, 16
    lay = split_lds(n_pad, (n + 63) // 64, m, 3, DC, 8 * 48, 8 * 64, 8, 163840)
    x = r * n_pad + np.where(b < n, inv[np.minimum(b, n - 1)], b)
    slot = np.where(x < lay["S"], lay["msg"] + 8 * x, -1)
    tval = (lay["zw"] + (n_pad // 64) * 8 + 15) & ~15
    wtab = lay["wtab"]
    tot = {"slot_read": 0, "slot_write": 0, "row_read2": 0, "wtab": 0}
    for t in range(nt):
        a = slot[t]
        tot["slot_read"] += sum(group_extra(a[g * 32:(g + 1) * 32][a[g * 32:(g + 1) * 32] >= 0], 64) for g in range(2))
        tot["slot_write"] += sum(group_extra(a[g * 16:(g + 1) * 16][a[g * 16:(g + 1) * 16] >= 0], 32) for g in range(4))
        row = tval + (t % NW) * (64 + DC) * 8
        p = np.arange(64) - start[t]
        for k in (0, 2, 4):
            for kk in (k, k + 1):
                ad = row + 8 * (start[t] + kk)
                tot["row_read2"] += sum(group_extra(ad[g * 16:(g + 1) * 16], 32) for g in range(4))
        wi = (deg[t] - 1) * DC + np.minimum(p, DC - 1)
        wa = wtab + wi * DC * 4
        for off, nb, gs in ((0, 32, 16), (8, 32, 16)):      # read2_b64: entries 0-1 and 2-3
            ad = wa + off
            tot["wtab"] += sum(group_extra(ad[g * gs:(g + 1) * gs], nb) for g in range(64 // gs))
        ad = wa + 16                                          # read_b64: entries 4-5
        tot["wtab"] += sum(group_extra(ad[g * 32:(g + 1) * 32], 64) for g in range(2))
    print(f"{nt} tasks; extra LDS cycles per task: " + ", ".join(f"{k} {v / nt:.2f}" for k, v in tot.items()))


if __name__ == "__main__":
    main()


def wtab_strides():
    """The weight-row reads' extra cycles per task against the row stride (dwords)."""
    n, m, nt, perm, b, r, chk, start, deg = plan_tasks()
    DC = 6
    for stride in (6, 8, 10, 12, 14):
        tot = 0
        for t in range(nt):
            p = np.arange(64) - start[t]
            wi = (deg[t] - 1) * DC + np.minimum(p, DC - 1)
            wa = wi * stride * 4
            for off in (0, 8):
                tot += sum(group_extra(wa[g * 16:(g + 1) * 16] + off, 32) for g in range(4))
            tot += sum(group_extra(wa[g * 32:(g + 1) * 32] + 16, 64) for g in range(2))
        print(f"wtab row stride {stride} dwords: {tot / nt:.2f} extra cycles per task")
