"""Checkpointed speculation (decode_split.hip, SPEC 2): decode time per batch
and restores across QBER and trigger (QKD_CKPT_UNSAT), against the exact
iterations (QKD_SPEC_CAP=0); results are checked equal to the exact ones.

    python tools/ckpt_sweep.py [frames]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import qkd_ldpc_amd as Q  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz")))
    H = Q.HMatrix.from_check_lists(int(g["dims"][0]), g["chk_off"], g["chk_idx"])
    seeds = torch.from_numpy(Q.make_seeds(99, F).view(np.int64)).cuda()
    caps = os.environ.get("CAPS", "8").split(",")
    trig = os.environ.get("TRIG", "8,16,32,64,128").split(",")
    for qn in [float(x) for x in os.environ.get("QS", "0.05,0.06,0.07,0.08,0.09").split(",")]:
        ws = Q.Workspace(H)
        alice, bob, eq = Q.keygen(H, seeds, qn, 0, workspace=ws)
        q = float(eq[0].item())

        def run(env):
            for k, v in env.items():
                Q.set_debug_option(k, v)
            outs = []
            Q.spec_replays(ws, reset=True)
            ts = []
            for _ in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = Q.qkd_ldpc(H, alice, bob, q, 50, 100.0, True, workspace=ws)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
                outs.append(r)
            for k in env:
                Q.set_debug_option(k, None)
            return outs[-1], float(np.median(ts[1:])), Q.spec_replays(ws, reset=True) / 4
        ref, t0, _ = run({"QKD_SPEC_CAP": "0"})
        rit = ref.iterations.cpu().numpy()
        print(f"q {q:.4f}: exact {t0:.3f} ms, mean it {rit.mean():.2f}, FER {1 - ref.keys_match.float().mean().item():.3f}",
              flush=True)
        for cap in caps:
            for tr in trig:
                r, t, n = run({"QKD_SPEC_CAP": cap, "QKD_CKPT_UNSAT": tr, "QKD_SPEC_CKPT": "1"})
                same = (r.iterations.cpu().numpy() == rit).all() and \
                    (r.keys_match.cpu() == ref.keys_match.cpu()).all() and \
                    (r.syndromes_match.cpu() == ref.syndromes_match.cpu()).all()
                print(f"  cap {cap} trigger {tr}: {t:.3f} ms ({t0 / t:.2f}x), restores/call {n:.0f}, "
                      f"same {bool(same)}", flush=True)


if __name__ == "__main__":
    main()
