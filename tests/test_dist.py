"""Frame sharding and the counter all-reduce of the multi-GPU path, on CPU with
gloo (world size 2), against a single-process reduction of the same frames."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from qkd_ldpc_amd.dist import allreduce_counters, shard_range


def test_shard_range_covers_every_frame_once():
    for frames in (1, 7, 4096, 1_000_000):
        for world in (1, 2, 3, 8):
            got = [shard_range(r, world, frames) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == frames
            for a, b in zip(got, got[1:]):
                assert a[1] == b[0]
            sizes = [e - b for b, e in got]
            assert max(sizes) - min(sizes) <= 1


def counters_of(iters, sp, ko):
    """qkd_counters bytes exactly as counters_kernel writes them."""
    it = iters[sp.astype(bool)].astype(np.uint64)
    rec = np.zeros(48, np.uint8)
    sums = np.array([len(iters), sp.sum(), (sp & ko).sum(), it.sum(), (it * it).sum()], np.uint64)
    rec[:40] = sums.view(np.uint8)
    ext = np.array([it.min() if it.size else 0xFFFFFFFF, it.max() if it.size else 0], np.uint32)
    rec[40:48] = ext.view(np.uint8)
    return rec


def _worker(rank, world, port, iters, sp, ko, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard_range(rank, world, len(iters))
    rec = torch.from_numpy(counters_of(iters[b:e], sp[b:e], ko[b:e]))
    allreduce_counters(rec)
    out[rank] = rec.numpy().tobytes()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_counter_allreduce_matches_single_process(world):
    rng = np.random.default_rng(0)
    f = 1001
    iters = rng.integers(2, 51, f).astype(np.uint32)
    sp = (rng.random(f) < 0.9).astype(np.uint8)
    ko = (rng.random(f) < 0.95).astype(np.uint8)
    sp[: f // 2] = 0                    # rank 0 sees no successful frame: min/max identities
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), iters, sp, ko, out), nprocs=world, join=True)
    want = counters_of(iters, sp, ko).tobytes()
    for r in range(world):
        assert out[r] == want
