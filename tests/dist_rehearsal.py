"""One rank of the multi-rank rehearsal (tests/test_dist.py): the launch,
sharding and counter all-reduce of bench.py's multi-GPU path (qkd_ldpc_amd.dist:
spawn_ranks -> init_rank -> shard_range -> allreduce_counters) over gloo on CPU,
with each rank's frames decoded by the oracle (test infrastructure; the GPU
path's own run is tests/test_dist_gpu.py). Usage (as a spawned rank):
    python tests/dist_rehearsal.py OUT_JSON FRAMES QBER [FAIL_RANK]
With QKD_REHEARSAL=point the ranks run bench.py's configs[3] path instead
(qkd_ldpc_amd.dist.run_sharded_point: untimed + timed shard runs, counter
all-reduce, max-rank time), the oracle decoding each shard.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    out, frames, q = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
    fail_rank = int(sys.argv[4]) if len(sys.argv) > 4 else -1
    import torch
    import torch.distributed as dist

    from qkd_ldpc_amd.dist import allreduce_counters, init_rank, rank_env, shard_range
    from oracle import oracle as O
    from test_dist import counters_of

    rank, world, local = rank_env()
    if rank == fail_rank:
        raise SystemExit(f"rank {rank}: failing on purpose")
    init_rank(world, local, backend="gloo", use_gpu=False)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz")))
    code = O.Code.from_lists(g)
    seeds = O.seeds(777, frames)
    if os.environ.get("QKD_REHEARSAL") == "point":
        from qkd_ldpc_amd.dist import run_sharded_point

        def run_shard(b, e):
            r = code.trials(q, seeds[b:e], 0, 50, 100.0, True, threads=2)
            return torch.from_numpy(counters_of(np.asarray(r["iters"], np.uint32),
                                                np.asarray(r["sp_ok"], np.uint8),
                                                np.asarray(r["key_ok"], np.uint8)))

        rec, dt, (b, e), per_rank = run_sharded_point(rank, world, frames, run_shard)
        t = torch.tensor([float(e - b)], dtype=torch.float64)
        dist.all_reduce(t)
        extra = {"seconds": dt, "per_rank_seconds": per_rank}
    else:
        b, e = shard_range(rank, world, frames)
        r = code.trials(q, seeds[b:e], 0, 50, 100.0, True, threads=2)
        rec = torch.from_numpy(counters_of(np.asarray(r["iters"], np.uint32), np.asarray(r["sp_ok"], np.uint8),
                                           np.asarray(r["key_ok"], np.uint8)))
        allreduce_counters(rec)
        t = torch.tensor([float(e - b)], dtype=torch.float64)
        dist.all_reduce(t)
        extra = {}
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"world": world, "counters": rec.numpy().tolist(), "frames": t.item(), **extra}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
