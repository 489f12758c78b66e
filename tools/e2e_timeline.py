"""One config-2 step of each bench path, for a kernel-trace timeline
(rocprofv3 --kernel-trace): 60 decode-only steps (qkd_qkd_ldpc_batch on
resident keys + qkd_counters_batch, as bench.py) then 60 end-to-end calls (qkd_trials_batch from the seeds),
with a 2 ms host sleep between the two groups as a marker.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/e2e_timeline.py
    python3 tools/e2e_timeline.py --summarise DIR/run_kernel_trace.csv
"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarise(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # split at the largest host gap (the marker sleep)
    gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"]), i) for i in range(len(rows) - 1)]
    cut = max(g for g in gaps if g[1] > 50)[1] + 1     # (past the set-up's first-call gaps)
    for name, grp in (("decode-only", rows[:cut]), ("end-to-end", rows[cut:])):
        # one step = from one decoder launch's predecessor run to the next; take the
        # last 20 steps, anchored on the split decoder
        dec = [i for i, r in enumerate(grp) if "decode_split_kernel" in r["Kernel_Name"]]
        steps = list(zip(dec[-21:-1], dec[-20:]))
        per = {}
        span = []
        for a, b in steps:
            t0 = int(grp[a]["Start_Timestamp"])
            span.append((int(grp[b]["Start_Timestamp"]) - t0) / 1e3)
            busy = 0
            for r in grp[a:b]:
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                per[k] = per.get(k, 0.0) + d / len(steps)
                busy += d
        ms = sum(span) / len(span)
        print(f"{name}: step {ms:.1f} us (decoder start to decoder start, mean of {len(steps)})")
        for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
            print(f"  {v:8.1f} us  {k}")
        print(f"  {ms - sum(per.values()):8.1f} us  gaps between kernels")


def main():
    import numpy as np
    import torch
    import qkd_ldpc_amd as Q
    from bench import load_code
    dev = torch.device("cuda", 0)
    H, _ = load_code(0)
    F, qb = 4096, 0.02
    seeds = torch.from_numpy(Q.make_seeds(777, F).view(np.int64)).to(dev)
    ws = Q.Workspace(H)
    alice, bob, eq = Q.keygen(H, seeds, qb, 0, workspace=ws)
    q = float(eq[0].item())
    iters = torch.empty(F, dtype=torch.int32, device=dev)
    sp = torch.empty(F, dtype=torch.uint8, device=dev)
    ko = torch.empty(F, dtype=torch.uint8, device=dev)
    counters = torch.empty(Q._native.COUNTERS_BYTES, dtype=torch.uint8, device=dev)
    L = Q._native.lib()
    sptr = int(torch.cuda.current_stream().cuda_stream)
    flags = Q.decoder_flags(True)
    for _ in range(60):          # bench.py's step: the decode call, then the counters
        Q._native.check(L.qkd_qkd_ldpc_batch(H.handle, ws.handle, alice.data_ptr(), bob.data_ptr(), F, q, 50,
                                             100.0, flags, None, iters.data_ptr(), sp.data_ptr(), ko.data_ptr(),
                                             sptr))
        Q._native.check(L.qkd_counters_batch(iters.data_ptr(), sp.data_ptr(), ko.data_ptr(), F,
                                             counters.data_ptr(), H.device, sptr))
    torch.cuda.synchronize()
    time.sleep(0.002)
    t = Q.run_trials(H, seeds, qb, 0, 50, 100.0, True, workspace=ws)
    for _ in range(60):
        Q.run_trials(H, seeds, qb, 0, 50, 100.0, True, workspace=ws, out=t)
    torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
        summarise(sys.argv[2])
    else:
        main()
