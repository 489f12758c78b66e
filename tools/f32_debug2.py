"""Debug aid: the binary32 sum-product model driven by the device's own tanhf /
atanhf (qkd_debug_math) against the kernel, per iteration cap, on one frame."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q
from qkd_ldpc_amd import _native as N
from oracle.variants import MinSumModel, sp_f32_decode
z = np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))
H = Q.HMatrix.from_check_lists(int(z["dims"][0]), z["chk_off"], z["chk_idx"])
M = MinSumModel(int(z["dims"][0]), int(z["dims"][1]), z["chk_off"], z["chk_idx"])

def dev_math(which):
    def f(v):
        x = torch.from_numpy(np.ascontiguousarray(v, np.float64).ravel()).cuda()
        y = torch.empty_like(x)
        N.check(N.lib().qkd_debug_math(which, x.data_ptr(), y.data_ptr(), x.numel(), None))
        torch.cuda.synchronize()
        return y.cpu().numpy().astype(np.float32).reshape(np.shape(v))
    return f

seeds = torch.from_numpy(Q.make_seeds(777, 1).view(np.int64)).cuda()
a, b, q = Q.keygen(H, seeds, 0.05, 4)
torch.cuda.synchronize()
A = a.cpu().numpy()
qq = float(q.cpu().numpy()[0])
lp = np.log((1 - qq) / qq)
llr = np.where(b.cpu().numpy() == 1, -lp, lp)
syn = M.syndrome(A)
tr = []
it, ok = sp_f32_decode(M, llr, syn, max_it=12, trace=tr, tanh_half=dev_math(2), two_atanh=dev_math(3),
                       trace_ref=A)
print(json.dumps({"model_dev_math": tr, "it": it.tolist(), "ok": ok.tolist()}))
tr2 = []
it, ok = sp_f32_decode(M, llr, syn, max_it=12, trace=tr2, trace_ref=A)
print(json.dumps({"model_np_math": tr2}))
