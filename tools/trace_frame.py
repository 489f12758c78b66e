"""Print one frame's decoder trace the way the reference's TRACE_SUM_PRODUCT /
TRACE_SUM_PRODUCT_LLR do (qkd_ldpc_algorithm.cpp:212-330), decoded on the GPU:

    python tools/trace_frame.py --alist FILE --seed S --qber Q [--max-iters 50] [--thr 100]
    python tools/trace_frame.py --dense FILE --alice 0110... --bob 0100... --qber Q

Keys come from the reference's per-trial generator (seed) or are given
literally; LLR = +-log((1-q)/q) with the exact QBER, syndrome = H alice.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q  # noqa: E402


def pr(name, arr, width=10):
    print(f"\n{name}:")
    for i in range(0, len(arr), width):
        print(" ".join(f"{x:g}" if isinstance(x, (float, np.floating)) else str(x) for x in arr[i:i + width]))


def main():
    ap = argparse.ArgumentParser()
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--alist")
    src.add_argument("--dense")
    ap.add_argument("--seed", type=int)
    ap.add_argument("--alice")
    ap.add_argument("--bob")
    ap.add_argument("--qber", type=float, required=True)
    ap.add_argument("--max-iters", type=int, default=50)
    ap.add_argument("--thr", type=float, default=100.0)
    ap.add_argument("--no-thr", action="store_true")
    args = ap.parse_args()
    H = Q.HMatrix.from_alist(args.alist) if args.alist else Q.HMatrix.from_dense(args.dense)
    n = H.num_bit_nodes
    if args.seed is not None:
        import torch
        seeds = torch.tensor([args.seed], dtype=torch.int64).cuda()
        a, b, q = Q.keygen(H, seeds, args.qber)
        alice, bob, q = a.cpu().numpy()[0], b.cpu().numpy()[0], float(q.cpu()[0])
    else:
        alice = np.array([int(c) for c in args.alice], np.uint8)
        bob = np.array([int(c) for c in args.bob], np.uint8)
        q = args.qber
    lp = np.log((1 - q) / q)
    llr = np.where(bob == 1, -lp, lp)
    cptr, cidx, _, _ = H.adjacency()
    syn = np.array([np.bitwise_xor.reduce(alice[cidx[cptr[j]:cptr[j + 1]]]) for j in range(H.num_check_nodes)])
    tr = Q.trace_decode(H, llr, syn, args.max_iters, args.thr, not args.no_thr)
    for t in range(tr["iterations"]):
        print(f"\n\nIteration: {t + 1}")
        pr("E", tr["E"][t])
        pr("L", tr["L"][t])
        pr("z", tr["z"][t])
        pr("s", tr["s"][t])
        if t < tr["M"].shape[0]:
            pr("M", tr["M"][t])
    print(f"\n\nMAX_LLR = {tr['max_llr']}")
    print(f"iterations {tr['iterations']}, syndromes match {tr['syndromes_match']}, n = {n}")


if __name__ == "__main__":
    main()
