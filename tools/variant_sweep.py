"""FER / iteration / time sweep of the decoder variants over BASELINE config 3's
QBER grid (alist N=10240, seed 777, 10,000 trials per point, <= 50 iterations).
Usage: python tools/variant_sweep.py [--trials T] [--scales 0.75,0.8125] > out.json"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--trials", type=int, default=10000)
ap.add_argument("--scales", default="0.75")
ap.add_argument("--variants", default="sp_f64,sp_f32,minsum")
args = ap.parse_args()

z = np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))
H = Q.HMatrix.from_check_lists(int(z["dims"][0]), z["chk_off"], z["chk_idx"])
seeds = torch.from_numpy(Q.make_seeds(777, args.trials).view(np.int64)).cuda()
grid = Q.qber_range(0.01, 0.09, 0.01)
runs = []
for v in args.variants.split(","):
    for sc in (args.scales.split(",") if v == "minsum" else [None]):
        runs.append((v, None if sc is None else float(sc)))
out = []
for v, sc in runs:
    for s, q in enumerate(grid):
        Q.run_trials(H, seeds[:64], q, s, variant=v, minsum_scale=sc)   # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = Q.run_trials(H, seeds, q, s, variant=v, minsum_scale=sc)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        c = Q.read_counters(r.counters)
        st = Q.counters_to_stats(c, args.trials, 50, q)
        rec = {"variant": v, "scale": sc, "qber": q, "fer": st["fer"],
               "mean_it": st["iterations_successful_sp_mean"],
               "sum_iters": int(c.sum_iters), "ms": dt * 1e3}
        out.append(rec)
        print(json.dumps(rec), flush=True)
