"""Multi-GPU sharding of a QBER point (frames are independent).

One process per GPU. Every rank derives the same seed stream
(simulation.cpp:222-228) and takes a contiguous frame range; nothing is
exchanged on the data path. The per-point counters of simulation.cpp:252-312
(frames, sp_ok, ldpc_ok, Σit, Σit², min it, max it) are combined with one
all-reduce each for the sums (SUM) and the extrema (MIN / MAX), over RCCL on
MI355X (backend "nccl") or gloo on CPU. The integer sums make the combined
mean/std independent of the rank count.
"""
from __future__ import annotations


def shard_range(rank: int, world: int, frames: int) -> tuple[int, int]:
    """[begin, end) of the frames rank `rank` decodes out of `frames` (balanced, contiguous)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(frames, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def allreduce_counters(counters, group=None):
    """In-place all-reduce of a qkd_counters record held as a uint8 tensor
    (layout of include/qkd_ldpc.h: 5 x uint64 sums, then uint32 min, uint32 max)."""
    import torch
    import torch.distributed as dist

    words = counters.view(torch.int64)              # 6 words: 5 sums + (min | max << 32)
    sums = words[:5]
    ext = counters[40:48].view(torch.int32)         # [min, max]
    mn = ext[0:1].to(torch.int64) & 0xFFFFFFFF      # uint32 -> non-negative int64
    mx = ext[1:2].to(torch.int64) & 0xFFFFFFFF
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    ext[0:1] = mn.to(torch.int32)                   # two's-complement store keeps the uint32 bits
    ext[1:2] = mx.to(torch.int32)
    return counters
