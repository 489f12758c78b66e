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


@pytest.mark.parametrize("world", [2, 3])
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


# ---- the launcher (qkd_ldpc_amd.dist.spawn_ranks / init_rank) and bench.py's use of it ----

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_spawned_ranks_reduce_to_single_rank_counters(tmp_path, oracle_mod, golden_code):
    """Two ranks started by spawn_ranks (the path `bench.py --gpus 2` takes without
    torchrun) shard 24 config-2 frames, decode their shares and all-reduce the counters
    over gloo: rank 0's record equals one process's record over all 24 frames."""
    from qkd_ldpc_amd.dist import spawn_ranks
    out = str(tmp_path / "r.json")
    frames, q = 24, 0.02
    rc = spawn_ranks(2, [os.path.join(ROOT, "tests", "dist_rehearsal.py"), out, str(frames), str(q)])
    assert rc == 0
    import json
    got = json.load(open(out))
    code = oracle_mod.Code.from_lists(golden_code)
    r = code.trials(q, oracle_mod.seeds(777, frames), 0, 50, 100.0, True, threads=2)
    want = counters_of(np.asarray(r["iters"], np.uint32), np.asarray(r["sp_ok"], np.uint8),
                       np.asarray(r["key_ok"], np.uint8))
    assert got["world"] == 2 and got["frames"] == frames
    assert bytes(got["counters"]) == want.tobytes()


def test_spawn_ranks_propagates_a_failed_rank(tmp_path):
    """A rank that dies makes the launcher fail (its peer, waiting in a collective,
    is terminated rather than left hanging)."""
    from qkd_ldpc_amd.dist import spawn_ranks
    rc = spawn_ranks(2, [os.path.join(ROOT, "tests", "dist_rehearsal.py"), str(tmp_path / "x.json"), "4",
                         "0.02", "1"])
    assert rc != 0


def _bench(args, env_extra=None, timeout=300):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus_disagreeing_with_world_size_fails():
    p = _bench(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0",
                                 "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29599"})
    assert p.returncode != 0 and "disagrees" in p.stderr


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure")
def test_bench_gpus_two_without_gpus_fails_loudly():
    """`bench.py --gpus 2` with no torchrun starts two ranks itself; here (no GPU) each
    rank must refuse to run rather than decode elsewhere."""
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert "no visible GPU" in p.stderr


def test_merge_counters_host_form():
    """dist.merge_counters on host records (the gloo path): sums add, min / max of the
    extrema, the identities of an all-failed record (UINT32_MAX / 0) neutral."""
    from qkd_ldpc_amd.dist import merge_counters
    rng = np.random.default_rng(3)
    recs = []
    for k in range(5):
        f = 50 + k
        it = rng.integers(2, 51, f).astype(np.uint32)
        sp = (rng.random(f) < (0.0 if k == 2 else 0.9)).astype(np.uint8)
        ko = (rng.random(f) < 0.9).astype(np.uint8)
        recs.append((it, sp, ko))
    rows = np.stack([counters_of(*r) for r in recs])
    out = torch.empty(48, dtype=torch.uint8)
    merge_counters(torch.from_numpy(rows), out)
    want = counters_of(np.concatenate([r[0] for r in recs]), np.concatenate([r[1] for r in recs]),
                       np.concatenate([r[2] for r in recs]))
    assert out.numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize("world", [2, 4])
def test_config4_point_over_ranks_matches_fixture(tmp_path, world):
    """bench.py's configs[3] path (dist.run_sharded_point: ONE all-gather of every
    rank's record and time) on 2 and 4 gloo ranks started by spawn_ranks, the oracle
    decoding each rank's shard of the first 40 config-4 frames: the merged record
    equals the config-4 fixture's counters over the same frames (bench.py
    config4_fixture_counters), and every rank's time is reported."""
    import json
    import sys
    from qkd_ldpc_amd.dist import spawn_ranks
    sys.path.insert(0, ROOT)
    from bench import config4_fixture_counters
    out = str(tmp_path / "c4.json")
    frames = 40
    rc = spawn_ranks(world, [os.path.join(ROOT, "tests", "dist_rehearsal.py"), out, str(frames), "0.02"],
                     env_extra={"QKD_REHEARSAL": "point"})
    assert rc == 0
    got = json.load(open(out))
    rec = np.array(got["counters"], np.uint8)
    sums = rec[:40].view(np.uint64)
    ext = rec[40:48].view(np.uint32)
    want = config4_fixture_counters(frames)
    assert got["frames"] == frames and got["seconds"] > 0 and got["world"] == world
    assert len(got["per_rank_seconds"]) == world and got["seconds"] >= max(got["per_rank_seconds"])
    assert [int(x) for x in sums] == [want["frames"], want["sp_ok"], want["ldpc_ok"], want["sum_iters"],
                                      want["sum_iters_sq"]]
    assert [int(ext[0]), int(ext[1])] == [want["min_iters"], want["max_iters"]]
