"""Step time against time since the first launch: consecutive blocks of B
config-2 steps (one qkd_qkd_ldpc_batch + counters each, as bench.py), each
block bracketed by synchronize, from a cold process. Shows whether the GPU's
clock ramps over the first tens of milliseconds of work.

    python tools/warm_probe.py [--blocks 40] [--block 5]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=40)
    ap.add_argument("--block", type=int, default=5)
    ap.add_argument("--sleep-ms", type=float, default=0.0, help="idle gap between blocks")
    args = ap.parse_args()
    import torch
    import qkd_ldpc_amd as Q
    import bench

    H, g = bench.load_code(torch.cuda.current_device())
    dev = torch.device("cuda", torch.cuda.current_device())
    F = 4096
    seeds = torch.from_numpy(Q.make_seeds(777, F).view(np.int64)).to(dev)
    ws = Q.Workspace(H)
    alice, bob, exact_q = Q.keygen(H, seeds, 0.02, 0, workspace=ws)
    q = float(exact_q[0].item())
    iters = torch.empty(F, dtype=torch.int32, device=dev)
    sp = torch.empty(F, dtype=torch.uint8, device=dev)
    ko = torch.empty(F, dtype=torch.uint8, device=dev)
    counters = torch.empty(Q._native.COUNTERS_BYTES, dtype=torch.uint8, device=dev)
    L = Q._native.lib()
    sptr = int(torch.cuda.current_stream().cuda_stream)
    flags = Q.decoder_flags(True, variant="sp_f64")

    def step():
        Q._native.check(L.qkd_qkd_ldpc_batch(H.handle, ws.handle, alice.data_ptr(), bob.data_ptr(), F, q, 50,
                                             100.0, flags, None, iters.data_ptr(), sp.data_ptr(), ko.data_ptr(),
                                             sptr))
        Q._native.check(L.qkd_counters_batch(iters.data_ptr(), sp.data_ptr(), ko.data_ptr(), F,
                                             counters.data_ptr(), H.device, sptr))

    torch.cuda.synchronize()
    t_start = time.perf_counter()
    rows = []
    for b in range(args.blocks):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.block):
            step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows.append(((t0 - t_start) * 1e3, (t1 - t0) * 1e3 / args.block))
        if args.sleep_ms:
            time.sleep(args.sleep_ms / 1e3)
    for t, ms in rows:
        print(f"t={t:8.2f} ms  step {ms:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
