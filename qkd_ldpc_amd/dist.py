"""Multi-GPU sharding of a QBER point (frames are independent).

One process per GPU. Every rank derives the same seed stream
(simulation.cpp:222-228) and takes a contiguous frame range; nothing is
exchanged on the data path. The per-point counters of simulation.cpp:252-312
(frames, sp_ok, ldpc_ok, Σit, Σit², min it, max it) are combined with ONE
collective per step: an all-gather of the 48-byte records (RCCL on MI355X,
backend "nccl"; gloo on CPU), then one merge launch on the device
(qkd_counters_merge: sums add, extrema min / max). The integer sums make the
combined mean/std independent of the rank count.

This replaces the reference's thread-pool fan-out of a point's trials
(simulation.cpp:230-250, `detach_loop` over THREADS_NUMBER threads): ranks
take the place of pool threads, a frame queue inside each rank's decoder the
place of the per-trial tasks.

Launching: `spawn_ranks` starts N copies of a script as ranks 0..N-1 (the
environment torchrun would give them: RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT) and makes no HIP call itself, so the
parent never initialises a GPU; `init_rank` is each rank's side: it checks the
world against the visible devices (one device per rank for RCCL; gloo may
share one), binds the device and opens the process group.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time


def shard_range(rank: int, world: int, frames: int) -> tuple[int, int]:
    """[begin, end) of the frames rank `rank` decodes out of `frames` (balanced, contiguous)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(frames, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


COUNTERS_BYTES = 48       # sizeof(qkd_counters), include/qkd_ldpc.h


def gather_records(rec, group=None):
    """One all-gather of every rank's `rec` (a 1-D tensor of the same size and
    dtype on every rank): returns a [world, rec.numel()] tensor, row r = rank r's
    record. The only collective of a step (RCCL on MI355X, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    src = rec.contiguous()
    if rec.is_cuda and dist.get_backend(group) == "gloo":
        src = src.cpu()              # gloo rehearsals on one device: host staging
    out = torch.empty(world * src.numel(), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.view(world, src.numel()).to(rec.device)


def merge_counters(records, out):
    """records: [n, 48] uint8 rows, each a qkd_counters record (include/qkd_ldpc.h:
    5 x uint64 sums, uint32 min, uint32 max) -> their combination in `out` (48
    bytes, may be a view of a row): sums add, extrema take min / max, the
    reduction of simulation.cpp:252-312 over the union of the ranks' frames.
    Device tensors: one qkd_counters_merge launch (the library's kernel) on the
    current stream. Host tensors (the gloo rehearsals on CPU): the same in numpy."""
    import numpy as np
    import torch

    n = records.shape[0]
    if records.is_cuda:
        from . import _native as N
        import ctypes

        recs = records.contiguous()
        N.check(N.lib().qkd_counters_merge(ctypes.c_void_p(recs.data_ptr()), n,
                                           ctypes.c_void_p(out.data_ptr()), out.device.index,
                                           ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)))
        return out
    a = records.contiguous().numpy().reshape(n, COUNTERS_BYTES)
    sums = a[:, :40].copy().view(np.uint64).sum(axis=0, dtype=np.uint64)
    ext = a[:, 40:48].copy().view(np.uint32)
    rec = np.zeros(COUNTERS_BYTES, np.uint8)
    rec[:40] = sums.view(np.uint8)
    rec[40:48] = np.array([ext[:, 0].min(), ext[:, 1].max()], np.uint32).view(np.uint8)
    out.copy_(torch.from_numpy(rec))
    return out


def allreduce_counters(counters, group=None):
    """In-place all-reduce of a qkd_counters record held as a uint8 tensor: ONE
    all-gather of the 48-byte records, then their merge on the device
    (qkd_counters_merge). Every rank ends with the same record."""
    merge_counters(gather_records(counters, group), counters)
    return counters


def run_sharded_point(rank: int, world: int, frames: int, run_shard, sync=None):
    """One QBER point of `frames` trials sharded over the ranks (BASELINE configs[3]:
    the reference's thread-pool fan-out of a point, simulation.cpp:230-250, and its
    reduction, :252-312).

    run_shard(begin, end) runs this rank's frames [begin, end) of the shared seed
    stream and returns its qkd_counters record (uint8 tensor, 48 bytes, on the
    rank's device). It is called twice: once untimed (allocation, clocks), then
    timed between a barrier + sync() on both sides. One all-gather then carries
    every rank's record and its own time: the records are merged (SUM / MIN /
    MAX) and the time is the max over ranks. Every rank must call this (it
    issues collectives when world > 1). Returns (counters, seconds, (begin,
    end), per_rank_seconds)."""
    import torch
    import torch.distributed as dist

    sync = sync or (lambda: None)
    b, e = shard_range(rank, world, frames)
    run_shard(b, e)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    counters = run_shard(b, e)
    sync()
    rank_dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    per_rank = [rank_dt]
    if world > 1:
        # [48-byte record | this rank's own time (binary64) | its barrier-inclusive time]
        rec = torch.empty(COUNTERS_BYTES + 16, dtype=torch.uint8, device=counters.device)
        rec[:COUNTERS_BYTES] = counters
        rec[COUNTERS_BYTES:] = torch.tensor([rank_dt, dt], dtype=torch.float64).view(torch.uint8).to(
            counters.device)
        g = gather_records(rec)
        merge_counters(g[:, :COUNTERS_BYTES], counters)
        t = g[:, COUNTERS_BYTES:].contiguous().view(torch.float64).view(world, 2).cpu()
        per_rank = [float(x) for x in t[:, 0]]
        dt = float(t[:, 1].max())
    return counters, dt, (b, e), per_rank


def rank_times(values, world):
    """All ranks' float values (e.g. their step time and decoder time) in one
    all-gather: returns a [world][len(values)] list (every rank gets it)."""
    import torch

    if world == 1:
        return [list(map(float, values))]
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    g = gather_records(torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev))
    return [[float(x) for x in row] for row in g.cpu()]


def imbalance(per_rank):
    """max / min of per-rank times (1.0 = perfectly balanced)."""
    lo = min(per_rank)
    return max(per_rank) / lo if lo > 0 else None


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(world: int, argv: list[str], env_extra: dict | None = None, poll_s: float = 0.2) -> int:
    """Run `python argv...` as ranks 0..world-1 on this node and wait for them.

    Each rank gets the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT). Their stdout/stderr
    are this process's. If one rank fails, the others (which would wait in a
    collective) are terminated, by their exact PIDs. Returns the first non-zero
    exit status, else 0. No GPU call is made here."""
    if world < 1:
        raise ValueError(f"world size must be >= 1, got {world}")
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    status = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc
                    for q in live:
                        q.terminate()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return status


def rank_env() -> tuple[int, int, int] | None:
    """(rank, world, local_rank) from a torchrun / spawn_ranks environment, or None."""
    if "WORLD_SIZE" not in os.environ:
        return None
    return (int(os.environ.get("RANK", "0")), int(os.environ["WORLD_SIZE"]),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_rank(world: int, local: int, backend: str | None = None, use_gpu: bool = True):
    """This rank's side of the launch: bind the device and open the process group.

    backend: "nccl" (RCCL, the default with a GPU) needs one visible device per
    rank on the node and fails loudly otherwise; "gloo" lets ranks share
    devices (local % visible) and runs without a GPU (use_gpu=False: CPU
    tensors, tests). Returns the torch.device this rank works on."""
    import torch
    import torch.distributed as dist

    backend = backend or os.environ.get("QKD_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if backend not in ("nccl", "gloo"):
        raise RuntimeError(f"QKD_DIST_BACKEND must be nccl or gloo, got {backend!r}")
    dev = torch.device("cpu")
    if use_gpu:
        n_dev = torch.cuda.device_count()
        if n_dev < 1:
            raise RuntimeError("no visible GPU for this rank")
        if backend == "nccl" and local >= n_dev:
            raise RuntimeError(f"world size {world}: local rank {local} has no GPU of its own "
                               f"({n_dev} visible; RCCL needs one device per rank, "
                               "QKD_DIST_BACKEND=gloo shares them)")
        dev = torch.device("cuda", local % n_dev)
        torch.cuda.set_device(dev)
    elif backend == "nccl":
        raise RuntimeError("the nccl (RCCL) backend needs GPUs")
    if world > 1 or backend == "nccl":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return dev
