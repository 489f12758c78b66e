"""Debug aid: frames where the binary32 sum-product variant fails at one QBER point."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import qkd_ldpc_amd as Q
z = np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))
H = Q.HMatrix.from_check_lists(int(z["dims"][0]), z["chk_off"], z["chk_idx"])
seeds = torch.from_numpy(Q.make_seeds(777, 10000).view(np.int64)).cuda()
r = Q.run_trials(H, seeds, 0.05, 4, variant="sp_f32")
torch.cuda.synchronize()
sp = r.syndromes_match.cpu().numpy(); ko = r.keys_match.cpu().numpy(); it = r.iterations.cpu().numpy()
bad = np.nonzero((sp == 0) | (ko == 0))[0]
print(json.dumps({"bad": bad[:40].tolist(), "it": it[bad[:40]].tolist(), "sp": sp[bad[:40]].tolist(),
                  "ko": ko[bad[:40]].tolist(), "n_bad": int(len(bad))}))
# per-iteration-cap outcome of the first bad frame through the LLR path
f = int(bad[0])
a, b, q = Q.keygen(H, seeds[f:f + 1], 0.05, 4)
torch.cuda.synchronize()
lp = np.log((1 - q.cpu().numpy()[0]) / q.cpu().numpy()[0])
llr = torch.where(b.to(torch.float64) == 1, -lp, lp).to(torch.float64).contiguous()
syn = Q.calculate_syndrome(H, a)
rows = []
for cap in range(1, 13):
    rr = Q.sum_product_decoding(H, llr, syn, cap, 100.0, True, variant="sp_f32")
    torch.cuda.synchronize()
    bits = rr.bits.cpu().numpy()[0]
    rows.append([cap, int(rr.iterations.cpu()[0]), int(rr.syndromes_match.cpu()[0]),
                 int((bits != a.cpu().numpy()[0]).sum())])
print(json.dumps({"frame": f, "caps": rows}))
