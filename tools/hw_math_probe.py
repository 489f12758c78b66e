import numpy as np, torch, sys
sys.path.insert(0, '/root/repo')
import qkd_ldpc_amd as Q
x = np.linspace(-120, 0, 2000001).astype(np.float32).astype(np.float64)
dx = torch.from_numpy(x).cuda(); dy = torch.empty_like(dx)
Q._native.check(Q._native.lib().qkd_debug_math(6, dx.data_ptr(), dy.data_ptr(), dx.numel(), None)); torch.cuda.synchronize()
y = dy.cpu().numpy(); ref = np.exp2(x)
rel = np.abs(y/ref - 1); k = np.argmax(rel)
print("exp2 max rel err", rel[k], "at", x[k], "ulp-ish", rel[k]/2**-24, "median", np.median(rel))
for lo, hi in [(-1,0),(-3,-1),(-10,-3),(-120,-10)]:
    m=(x>=lo)&(x<hi); print(" range", lo, hi, rel[m].max()/2**-24)
x = np.exp(np.linspace(np.log(1e-30), np.log(3.0), 2000001)).astype(np.float32).astype(np.float64)
dx = torch.from_numpy(x).cuda(); dy = torch.empty_like(dx)
Q._native.check(Q._native.lib().qkd_debug_math(7, dx.data_ptr(), dy.data_ptr(), dx.numel(), None)); torch.cuda.synchronize()
y = dy.cpu().numpy(); ref = np.log2(x)
ab = np.abs(y - ref); k = np.argmax(ab)
print("log2 max abs err", ab[k], "at", x[k], "= 2^", np.log2(ab[k]))
rel = ab/np.maximum(np.abs(ref),1e-300)
for lo, hi in [(1e-30,0.5),(0.5,0.9),(0.9,1.1),(1.1,2),(2,3)]:
    m=(x>=lo)&(x<hi); print(" range", lo, hi, "max abs", ab[m].max(), "max rel", rel[m].max())
