"""FER of min-sum settings (scale, offset) against the reference decoder (sp_f64) and
the binary32 sum-product variant on BASELINE config 3's hardest points, on one GPU.

    python tools/minsum_sweep.py [--trials 100000] [--qbers 0.07,0.08] > out.jsonl

Frames k < trials of point s use seeds 777[k] + s (s = 6 for 0.07, 7 for 0.08, as in
config 3). Prints one JSON line per (decoder, setting, QBER)."""
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
ap.add_argument("--trials", type=int, default=100000)
ap.add_argument("--qbers", default="0.07,0.08")
ap.add_argument("--scales", default="0.75,0.8125,0.875,0.9375,1.0")
ap.add_argument("--offsets", default="0,0.125,0.25,0.375,0.5")
ap.add_argument("--self-correct", default="0", help="comma list of 0/1: plain and/or self-corrected min-sum")
args = ap.parse_args()

z = np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))
H = Q.HMatrix.from_check_lists(int(z["dims"][0]), z["chk_off"], z["chk_idx"])
seeds = torch.from_numpy(Q.make_seeds(777, args.trials).view(np.int64)).cuda()
grid = Q.qber_range(0.01, 0.09, 0.01)
runs = [("sp_f64", None, None, False), ("sp_f32", None, None, False)]
for scm in args.self_correct.split(","):
    for sc in args.scales.split(","):
        for of in args.offsets.split(","):
            runs.append(("minsum", float(sc), float(of) if float(of) > 0 else None, scm == "1"))
for q in [float(x) for x in args.qbers.split(",")]:
    s = min(range(len(grid)), key=lambda k: abs(grid[k] - q))
    for v, sc, of, scm in runs:
        kw = {} if v != "minsum" else {"minsum_scale": None if sc == 1.0 else sc, "minsum_offset": of,
                                      "minsum_self_correct": scm}
        if v == "minsum" and sc == 1.0:
            kw["minsum_scale"] = 255 / 256
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = Q.run_trials(H, seeds, grid[s], s, variant=v, **kw)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        st = Q.counters_to_stats(Q.read_counters(r.counters), args.trials, 50, grid[s])
        print(json.dumps({"variant": v, "scale": kw.get("minsum_scale"), "offset": of, "self_correct": scm,
                          "qber": grid[s],
                          "trials": args.trials, "fer": st["fer"],
                          "mean_it": st["iterations_successful_sp_mean"], "ms": dt * 1e3}), flush=True)
