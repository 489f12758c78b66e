"""Can one trial call hide its key generation by splitting into chunks on two
streams? (end to end; round-6 verdict item 6)

Times, on one GPU, K config-2 steps of 4096 frames of fused trials
(qkd_trials_batch: keygen + frame syndromes + decode + counters):
  one     one call of 4096 frames (stream A)
  chunksC the frames in C chunks, chunk k on stream A (k even) or B (k odd),
          each with its own workspace; a step starts both streams together and
          ends when both are done (an event join), so steps do not overlap
Each chunk's decoder can fill the previous chunk's tail, and its key
generation can run beside the other stream's work.

    python tools/chunk_probe.py [K]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q  # noqa: E402
from bench import load_code  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    H, _ = load_code(0)
    F, qb = 4096, 0.02
    seeds = torch.from_numpy(Q.make_seeds(777, F).view(np.int64)).to(dev)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ws = [Q.Workspace(H) for _ in range(4)]
    out = {}

    def one():
        with torch.cuda.stream(sa):
            out["one"] = Q.run_trials(H, seeds, qb, 0, 50, workspace=ws[0], stream=sa, out=out.get("one"))

    def chunks(C):
        step = F // C
        start = torch.cuda.Event()
        start.record(sa)
        sb.wait_event(start)
        for k in range(C):
            s = sa if k % 2 == 0 else sb
            key = f"c{C}_{k}"
            with torch.cuda.stream(s):
                out[key] = Q.run_trials(H, seeds[k * step:(k + 1) * step], qb, 0, 50, workspace=ws[k % 4],
                                        stream=s, out=out.get(key))
        end = torch.cuda.Event()
        end.record(sb)
        sa.wait_event(end)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / K

    cases = {"one": one, "chunks2": lambda: chunks(2), "chunks4": lambda: chunks(4)}
    for _ in range(3):
        for fn in cases.values():
            timed(fn)
    r = {}
    for rep in range(3):
        for name, fn in cases.items():
            r.setdefault(name, []).append(timed(fn))
    for k, v in r.items():
        print(f"{k:8s} ms per step: " + " ".join(f"{x:.4f}" for x in v), flush=True)
    # the chunked runs decode the same frames: same outcomes
    it1 = out["one"].iterations.cpu()
    for C in (2, 4):
        itc = torch.cat([out[f"c{C}_{k}"].iterations.cpu() for k in range(C)])
        print(f"chunks{C} iterations equal: {bool(torch.equal(it1, itc))}")


if __name__ == "__main__":
    main()
