"""A rank for tests/test_dist_gpu.py: opens an RCCL ("nccl") process group on the
MI355X through qkd_ldpc_amd.dist.init_rank and all-reduces real counter records
produced by qkd_trials_batch / qkd_counters_batch. Usage (as a spawned rank):
    python tests/dist_gpu_rank.py OUT_JSON
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    import torch
    import torch.distributed as dist

    from qkd_ldpc_amd.dist import allreduce_counters, init_rank, rank_env

    rank, world, local = rank_env()
    dev = init_rank(world, local, backend="nccl")
    assert dist.get_backend() == "nccl"
    import qkd_ldpc_amd as Q

    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz")))
    H = Q.HMatrix.from_check_lists(int(g["dims"][0]), g["chk_off"], g["chk_idx"], device=dev.index)
    seeds = torch.from_numpy(Q.make_seeds(777, 512).view(np.int64)).to(dev)
    r = Q.run_trials(H, seeds, 0.02)
    before = r.counters.clone()
    allreduce_counters(r.counters)
    torch.cuda.synchronize()
    same_ok = bool(torch.equal(before, r.counters))
    # an all-failed shard: no successful frame, min/max at their identities
    it = torch.full((64,), 50, dtype=torch.int32, device=dev)
    zero = torch.zeros(64, dtype=torch.uint8, device=dev)
    c = torch.empty(Q._native.COUNTERS_BYTES, dtype=torch.uint8, device=dev)
    Q._native.check(Q._native.lib().qkd_counters_batch(it.data_ptr(), zero.data_ptr(), zero.data_ptr(), 64,
                                                       c.data_ptr(), dev.index, None))
    torch.cuda.synchronize()
    before_f = c.clone()
    allreduce_counters(c)
    torch.cuda.synchronize()
    ext = c[40:48].cpu().numpy().view(np.uint32)
    res = {"world": world, "backend": dist.get_backend(), "same_ok": same_ok,
           "same_failed": bool(torch.equal(before_f, c)), "failed_minmax": [int(ext[0]), int(ext[1])],
           "counters": r.counters.cpu().numpy().tolist()}
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
