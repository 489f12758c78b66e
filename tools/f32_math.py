"""Debug aid: the binary32 variant's device tanh(x/2) / 2 atanh(x) against numpy float32."""
import os, sys, json
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qkd_ldpc_amd import _native as N
x = np.concatenate([np.linspace(-100, 100, 200001), np.linspace(-1, 1, 200001),
                    np.array([0.0, -0.0, 1.0, -1.0, 88.0, 89.0, 100.0, -100.0, 1e-30, 1e-40])])
xd = torch.from_numpy(x).cuda()
out = {}
for which, name, ref in [(2, "tanh_half", lambda v: np.tanh(v.astype(np.float32) * np.float32(0.5))),
                         (3, "two_atanh", lambda v: np.float32(2) * np.arctanh(np.clip(v.astype(np.float32), -np.float32(0x1.fffffep-1), np.float32(0x1.fffffep-1))))]:
    y = torch.empty_like(xd)
    N.check(N.lib().qkd_debug_math(which, xd.data_ptr(), y.data_ptr(), x.size, None))
    torch.cuda.synchronize()
    g = y.cpu().numpy()
    with np.errstate(all="ignore"):
        w = ref(x).astype(np.float64)
    nan_g = np.isnan(g); nan_w = np.isnan(w)
    fin = np.isfinite(g) & np.isfinite(w)
    rel = np.abs(g[fin] - w[fin]) / np.maximum(np.abs(w[fin]), 1e-30)
    out[name] = {"nan_dev": int(nan_g.sum()), "nan_np": int(nan_w.sum()),
                 "nan_dev_x": x[nan_g & ~nan_w][:10].tolist(),
                 "inf_mismatch": int((np.isinf(g) != np.isinf(w)).sum()),
                 "max_rel": float(rel.max()), "ulp_gt1": int((rel > 2.4e-7).sum())}
print(json.dumps(out))
