"""Throughput of the large-code path (totals in global memory): a random
(3,6)-regular code of N bits, F frames of fused trials at one QBER."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import qkd_ldpc_amd as Q  # noqa: E402
from test_large_codes import regular_code  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=40000)
ap.add_argument("--frames", type=int, default=4096)
ap.add_argument("--qber", type=float, default=0.03)
ap.add_argument("--variant", default="sp_f64")
ap.add_argument("--phase-timing", action="store_true", help="per-phase shader clocks (QKD_PHASE_TIMING option)")
ap.add_argument("--debug-opt", action="append", default=[], metavar="NAME=VALUE",
                help="a library debug option (qkd_debug_set_option), process-wide; repeatable")
args = ap.parse_args()
for kv in args.debug_opt + (["QKD_PHASE_TIMING=1"] if args.phase_timing else []):
    Q.set_debug_option(kv.partition("=")[0], kv.partition("=")[2])
m, cp, ci = regular_code(args.n, seed=11)
H = Q.HMatrix.from_check_lists(args.n, cp, ci)
seeds = torch.from_numpy(Q.make_seeds(777, args.frames).view(np.int64)).cuda()
ws = Q.Workspace(H)
a, b, q = Q.keygen(H, seeds, args.qber)
Q.qkd_ldpc(H, a, b, float(q[0]), 50, variant=args.variant, workspace=ws)
torch.cuda.synchronize()
t = time.perf_counter()
steps = 5
for _ in range(steps):
    r = Q.qkd_ldpc(H, a, b, float(q[0]), 50, variant=args.variant, workspace=ws)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / steps
it = r.iterations.cpu().numpy()
# lockstep model of a frame-interleaved store: g frames decoded
# together run as long as their slowest; without refill a batch costs the sum
# over groups of the group maximum, against the sum of the frames' own counts
hist = np.bincount(it).tolist()
lock = {str(g): float(it[: len(it) // g * g].reshape(-1, g).max(axis=1).sum() * g / it[: len(it) // g * g].sum())
        for g in (2, 4, 8, 16)}
extra = {}
if args.phase_timing:
    # the last call's summed shader-clock cycles per phase (the interleaved
    # decoder: check, bit, syndrome test + outcomes, refill)
    cyc = np.zeros(7, dtype=np.uint64)
    Q._native.check(Q._native.lib().qkd_debug_phase_cycles(ws.handle, cyc.ctypes.data))
    tot = float(cyc.sum())
    extra["phase_cycles"] = cyc.tolist()
    extra["phase_share"] = [round(float(x) / tot, 4) for x in cyc] if tot else []
print(json.dumps({**extra, "n": args.n, "m": m, "frames": args.frames, "qber": args.qber, "variant": args.variant,
                  "ms_per_batch": dt * 1e3, "gbit_s": args.frames * args.n / dt / 1e9,
                  "mean_it": float(it.mean()), "iter_hist": hist, "max_it": int(it.max()),
                  "lockstep_work_ratio": lock, "fer": float(1 - r.keys_match.cpu().numpy().mean())}))
