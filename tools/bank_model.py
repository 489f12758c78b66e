"""LDS bank model of the split decoder's check phases (CPU, no GPU): for the
N=10240 code, the wave plan (a port of qkd_plan.h build_wave_plan), the internal
bit order (host.cpp build_code) and an LDS slot budget S, count per task and
half-wave the LDS slot accesses (x = row * n_pad + bit < S) that share a bank pair
(x mod 32, 8-byte slots over 64 four-byte banks) with a different slot: the extra
cycles a ds_read_b64 / ds_write_b64 of that half-wave costs. Also the number of
distinct 128-byte lines the global slots (x >= S) of each task touch.

    python tools/bank_model.py [S]
"""
import sys

import numpy as np


def build_plan(n, m, cptr, cidx, krow):
    by_deg = {}
    for j in range(m):
        by_deg.setdefault(cptr[j + 1] - cptr[j], []).append(j)
    degs = sorted(by_deg, reverse=True)
    nxt = {d: 0 for d in degs}
    left = m
    words = []
    while left > 0:
        reach = [{0: None}]
        for d in degs:
            avail = len(by_deg[d]) - nxt[d]
            r2 = {}
            for c in reach[-1]:
                for x in range(min(avail, (64 - c) // d), -1, -1):
                    if c + x * d not in r2:
                        r2[c + x * d] = x
            reach.append(r2)
        best = max(reach[-1])
        cnt = [0] * len(degs)
        c = best
        for i in range(len(degs), 0, -1):
            cnt[i - 1] = reach[i][c]
            c -= cnt[i - 1] * degs[i - 1]
        task = [(n, 0)] * 64
        lane = 0
        for i, d in enumerate(degs):
            for _ in range(cnt[i]):
                j = by_deg[d][nxt[d]]
                nxt[d] += 1
                left -= 1
                for k in range(d):
                    task[lane + k] = (int(cidx[cptr[j] + k]), int(krow[cptr[j] + k]))
                lane += d
        words.append(task)
    return words


def main():
    g = np.load("tests/golden/code_n10240.npz")
    n, m = int(g["dims"][0]), int(g["dims"][1])
    cptr, cidx = g["chk_off"].astype(int), g["chk_idx"].astype(int)
    bdeg = np.bincount(cidx, minlength=n)
    fill = np.zeros(n, int)
    krow = np.zeros(len(cidx), int)
    for j in range(m):
        for k in range(cptr[j], cptr[j + 1]):
            b = cidx[k]
            krow[k] = fill[b]
            fill[b] += 1
    plan = build_plan(n, m, cptr, cidx, krow)
    n_pad = (n + 1 + 63) // 64 * 64
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 18432
    inv = -np.ones(n, int)
    nx = 0
    for task in plan:
        for b, r in task:
            if b < n and r == bdeg[b] - 1 and inv[b] < 0:
                inv[b] = nx
                nx += 1
    for name, order in (("original", np.arange(n)), ("internal", inv)):
        extra = lines = acc = 0
        for task in plan:
            xs = [r * n_pad + (order[b] if b < n else n) for b, r in task]
            for h in (xs[:32], xs[32:]):
                lds = sorted(set(x for x in h if x < S))
                acc += len(lds)
                banks = {}
                for x in lds:
                    banks[x % 32] = banks.get(x % 32, 0) + 1
                extra += max(banks.values()) - 1 if banks else 0
            lines += len(set((x - S) * 8 // 128 for x in xs if x >= S))
        t = len(plan)
        print(f"{name}: {t} tasks, LDS accesses/task {acc / t:.1f}, extra bank cycles/task "
              f"{extra / t:.2f}, global 128-B lines/task {lines / t:.2f}")


if __name__ == "__main__":
    main()
