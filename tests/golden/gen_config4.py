"""Generate tests/golden/config4_1m.npz: BASELINE config 4 per frame, from the oracle.

Config 4 is config 2's parameters (alist N=10240, SIMULATION_SEED 777, QBER 0.02,
<= 50 iterations, clamp 100) with TRIALS_NUMBER = 1,000,000:
frame k is seeded seeds[k] + 0, seeds[k] the k-th xoshiro256++(777) draw
(simulation.cpp:222-228, :247). The reference shards nothing; the 8-GPU run gives
rank r the frames [r F/8, (r+1) F/8) and all-reduces the counters.

Runs here or anywhere the oracle builds (needs only tests/golden/code_n10240.npz):

    python tests/golden/gen_config4.py [--frames 1000000] [--threads 8]

Outputs (data only):
  iters   uint8[F]   iterations_num of every frame (1..50)
  sp      packed bits, syndromes_match;  ko  packed bits, keys_match
  exact_q float64    initial_QBER (equal for every frame: floor(N q) / N)
  stats   json       the simulation.cpp:252-312 reduction of all F frames
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=os.path.join(HERE, "config4_1m.npz"))
    args = ap.parse_args()
    O.build()
    code = O.Code.from_lists(dict(np.load(os.path.join(HERE, "code_n10240.npz"))))
    seeds = O.seeds(777, args.frames)
    iters = np.zeros(args.frames, np.uint8)
    sp = np.zeros(args.frames, bool)
    ko = np.zeros(args.frames, bool)
    q0 = None
    chunk = 50_000
    t0 = time.time()
    for b in range(0, args.frames, chunk):
        e = min(args.frames, b + chunk)
        r = code.trials(0.02, seeds[b:e], 0, 50, 100.0, True, threads=args.threads)
        iters[b:e] = r["iters"]
        sp[b:e] = r["sp_ok"]
        ko[b:e] = r["key_ok"]
        assert (r["exact_q"] == r["exact_q"][0]).all()
        q0 = float(r["exact_q"][0])
        print(f"{e} frames, {time.time() - t0:.0f} s", flush=True)
    st = O.batch_stats(iters, sp, ko, np.array([q0]), args.frames, 50)
    st["frames"] = args.frames
    st["sum_iters_sq_sp"] = int((iters[sp].astype(np.int64) ** 2).sum())
    st["oracle_seconds"] = round(time.time() - t0, 1)
    st["oracle_threads"] = args.threads
    print(json.dumps(st))
    np.savez_compressed(args.out, iters=iters, sp=np.packbits(sp), ko=np.packbits(ko),
                        exact_q=np.array([q0]), stats=np.array(json.dumps(st)))
    print("wrote", args.out)


if __name__ == "__main__":
    main()
