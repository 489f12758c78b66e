"""The interleaved decoder (QKD_ILV=1) against the split kernel (QKD_ILV=0) on
a random (3,6) code of N bits: iterations, syndrome and key flags equal.

    python tools/ilv_equal_check.py N [frames] [qber]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import qkd_ldpc_amd as Q  # noqa: E402
from test_large_codes import regular_code  # noqa: E402

n = int(sys.argv[1])
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
qb = float(sys.argv[3]) if len(sys.argv) > 3 else 0.02
m, cp, ci = regular_code(n, seed=11)
H = Q.HMatrix.from_check_lists(n, cp, ci)
seeds = torch.from_numpy(Q.make_seeds(2024, frames).view(np.int64)).cuda()
a, b, q = Q.keygen(H, seeds, qb)
out = {}
for mode in ("1", "0"):
    Q.set_debug_option("QKD_ILV", mode)
    r = Q.qkd_ldpc(H, a, b, float(q[0]), 50)
    torch.cuda.synchronize()
    out[mode] = r
x, y = out["1"], out["0"]
ok = (torch.equal(x.iterations, y.iterations) and torch.equal(x.syndromes_match, y.syndromes_match)
      and torch.equal(x.keys_match, y.keys_match))
print(f"n={n} frames={frames} qber={qb} equal={ok} mean_it={x.iterations.float().mean().item():.3f}")
sys.exit(0 if ok else 1)
