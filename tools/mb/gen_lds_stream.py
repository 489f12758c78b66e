"""Address streams of the split decoder's LDS accesses for tools/mb/lds_bank_mb.hip
(config 2: the N = 10240 code, the speculative keys-path layout). Writes
tools/mb/lds_stream.bin:
  u32 n_tasks, u32 n_bits, then
  check-phase slot words: n_tasks * 64 u32 LDS byte addresses (a global slot:
      0x40000 + its byte offset in the region, an address past the allocation,
      as the kernel's encoded words give the LDS half of the access),
  bit-phase syndrome words: n_pad * 3 u32 byte addresses of xsyn words of the
      internal bit's three checks.
The layout (S, msg) is SplitLds's (qkd_decode.h) for DC = 6, tab2 = 8 patterns x
48 entries, ftab = 8 x 64 entries, budget 163840.

    python tools/mb/gen_lds_stream.py
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def split_lds(n_pad, n_words, m, max_dv, dc, tab2_entries, ftab_entries, esz, budget):
    m_words = ((m + 63) // 64) * 2
    a16 = lambda x: (x + 15) & ~15
    tsyn = 0
    qsyn = tsyn + m_words * 4
    xsyn = qsyn + m_words * 4
    zw = a16(xsyn + m_words * 8)
    tval = a16(zw + (n_pad // 64) * 8)
    rows = 16 * (64 + dc) * esz
    stage = n_words * 16
    ctab = a16(tval + max(rows, stage))
    tab2 = ctab + 17 * 8
    ftab = a16(tab2 + tab2_entries * 8)
    ctl = a16(ftab + ftab_entries * 8)
    wtab = ctl + 32
    msg = a16(wtab + (dc * dc * dc if dc <= 8 else 0) * 4)
    slots = max_dv * n_pad
    fit = (budget - msg) // esz - 64 if budget > msg + 64 * esz else 0
    S = min(slots, fit) & ~63
    return dict(xsyn=xsyn, msg=msg, S=S, zw=zw, wtab=wtab)


def main():
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
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    n_pad = (n + 1 + 63) // 64 * 64
    lay = split_lds(n_pad, (n + 63) // 64, m, 3, 6, 8 * 48, 8 * 64, 8, 163840)
    b = (plan & 0xFFFFFF).astype(np.int64)
    row = (plan >> 24).astype(np.int64)
    x = row * n_pad + np.where(b < n, inv[np.minimum(b, n - 1)], b)
    addr = np.where(x < lay["S"], lay["msg"] + 8 * x, 0x40000 + 8 * (x - lay["S"])).astype(np.uint32)
    # xsyn words of each internal bit's checks (ascending)
    chk = np.zeros((n_pad, 3), np.int64)
    deg = np.zeros(n, np.int64)
    for j in range(m):
        for k in range(cptr[j], cptr[j + 1]):
            bb = cidx[k]
            chk[inv[bb], deg[bb]] = j
            deg[bb] += 1
    syn = (lay["xsyn"] + 4 * (chk >> 5)).astype(np.uint32)
    out = os.path.join(ROOT, "tools", "mb", "lds_stream.bin")
    with open(out, "wb") as f:
        np.array([nt.value, n_pad], np.uint32).tofile(f)
        addr.tofile(f)
        syn.tofile(f)
    glob = (x >= lay["S"]).mean()
    print(f"{out}: {nt.value} tasks, S={lay['S']} msg={lay['msg']}, {glob:.3f} of check-phase lanes global")


if __name__ == "__main__":
    main()
