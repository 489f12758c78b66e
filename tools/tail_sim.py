"""Frame-order experiment for the decoder's frame queue: per-frame iteration
counts of a bench batch (config 2) against the initial syndrome mismatch weight
|H a xor H b|, and a simulated dynamic queue of W workgroups (frame time
a + iterations) in seed order, weight-descending order and iteration-descending
order (the ideal).

    python tools/tail_sim.py [--frames 4096] [--qber 0.02] [--workers 256]"""
import argparse
import heapq
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=4096)
ap.add_argument("--qber", type=float, default=0.02)
ap.add_argument("--workers", type=int, default=256)
ap.add_argument("--overhead", type=float, default=1.0, help="per-frame cost in iterations")
args = ap.parse_args()

z = np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))
H = Q.HMatrix.from_check_lists(int(z["dims"][0]), z["chk_off"], z["chk_idx"])
seeds = torch.from_numpy(Q.make_seeds(777, args.frames).view(np.int64)).cuda()
a, b, qx = Q.keygen(H, seeds, args.qber, 0)
r = Q.qkd_ldpc(H, a, b, float(qx[0].item()), 50, 100.0, True)
torch.cuda.synchronize()
it = r.iterations.cpu().numpy().astype(np.int64)
A = a.cpu().numpy().astype(np.int64)
B = b.cpu().numpy().astype(np.int64)
off, idx = z["chk_off"], z["chk_idx"]
Hs = sp.csr_matrix((np.ones(idx.size, np.int64), idx, off), shape=(off.size - 1, A.shape[1]))
w = np.asarray((Hs @ (A ^ B).T) & 1).sum(axis=0)
err = (A ^ B).sum(axis=1)


def makespan(order, cost):
    heap = [0.0] * args.workers
    for f in order:
        t = heapq.heappop(heap)
        heapq.heappush(heap, t + cost[f])
    return max(heap)


cost = it + args.overhead
tot = cost.sum() / args.workers
out = {
    "frames": args.frames, "qber": args.qber, "mean_it": float(it.mean()), "max_it": int(it.max()),
    "it_hist": np.bincount(it).tolist(),
    "corr_weight_it": float(np.corrcoef(w, it)[0, 1]), "corr_errors_it": float(np.corrcoef(err, it)[0, 1]),
    "lower_bound": float(tot),
    "seed_order": makespan(range(args.frames), cost),
    "weight_desc": makespan(np.argsort(-w, kind="stable"), cost),
    "iters_desc": makespan(np.argsort(-it, kind="stable"), cost),
}
print(json.dumps(out))
