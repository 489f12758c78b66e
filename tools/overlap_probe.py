"""Can key generation run beside the decoder? (end to end)

Times, on one GPU, K config-2 batches of
  decode  qkd_qkd_ldpc_batch on resident keys (stream A, workspace 1)
  keygen  qkd_keygen_batch of other frames (stream B, workspace 2)
alone, one after the other, and issued together on the two streams with no
dependency between them. If the decoder's persistent workgroups leave no room
(VGPRs / LDS / wave slots), "together" equals "sequential".

    python tools/overlap_probe.py [K]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q  # noqa: E402
from bench import load_code, VARIANTS  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    H, _ = load_code(0)
    F, qb = 4096, 0.02
    seeds = torch.from_numpy(Q.make_seeds(777, 2 * F).view(np.int64)).to(dev)
    ws1, ws2 = Q.Workspace(H), Q.Workspace(H)
    alice, bob, eq = Q.keygen(H, seeds[:F], qb, 0, workspace=ws1)
    q = float(eq[0].item())
    L = Q._native.lib()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    iters = torch.empty(F, dtype=torch.int32, device=dev)
    sp = torch.empty(F, dtype=torch.uint8, device=dev)
    ko = torch.empty(F, dtype=torch.uint8, device=dev)
    n = H.num_bit_nodes
    ka = torch.empty((F, n), dtype=torch.uint8, device=dev)
    kb = torch.empty_like(ka)
    kq = torch.empty(F, dtype=torch.float64, device=dev)
    flags = Q.decoder_flags(True, **VARIANTS["sp_f64"])

    def dec():
        Q._native.check(L.qkd_qkd_ldpc_batch(H.handle, ws1.handle, alice.data_ptr(), bob.data_ptr(), F, q, 50, 100.0,
                                             flags, None, iters.data_ptr(), sp.data_ptr(), ko.data_ptr(),
                                             int(sa.cuda_stream)))

    def kg():
        Q._native.check(L.qkd_keygen_batch(H.handle, ws2.handle, seeds[F:].data_ptr(), 0, F, qb, ka.data_ptr(),
                                           kb.data_ptr(), kq.data_ptr(), int(sb.cuda_stream)))

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / K

    for _ in range(3):
        timed(dec)
        timed(kg)
    r = {}
    for rep in range(3):
        r.setdefault("decode", []).append(timed(dec))
        r.setdefault("keygen", []).append(timed(kg))
        r.setdefault("together", []).append(timed(lambda: (dec(), kg())))
    for k, v in r.items():
        print(f"{k:9s} ms per batch: " + " ".join(f"{x:.4f}" for x in v))
    d, g, t = (min(r[k]) for k in ("decode", "keygen", "together"))
    print(f"hidden share of keygen: {(d + g - t) / g:.2f}")


if __name__ == "__main__":
    main()
