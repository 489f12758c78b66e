"""Key-generator probe for counter passes: config-2 keys (4096 frames, QBER 0.02)
generated N times on the device (keygen_split_kernel), nothing else.

    rocprofv3 --pmc ... -- python3 tools/kg_probe.py [N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q  # noqa: E402
from bench import load_code  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
H, _ = load_code(0)
seeds = torch.from_numpy(Q.make_seeds(777, 4096).view(np.int64)).cuda()
ws = Q.Workspace(H)
for _ in range(n):
    Q.keygen(H, seeds, 0.02, 0, workspace=ws)
torch.cuda.synchronize()
print("ok")
