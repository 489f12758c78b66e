"""BASELINE config 4: C2 parameters with 1,000,000 frames, sharded over 8 ranks
(simulation.cpp:192-316, seeds :222-228, reduction :252-312).

The fixture tests/golden/config4_1m.npz holds the oracle's per-frame results for all
1M frames (tests/golden/gen_config4.py). On one MI355X the 8 ranks' shares run as
eight 125,000-frame qkd_trials_batch launches over shard_range; every frame must
match, the summed shard counters must equal one 1M-frame launch's counters, and the
statistics must equal the oracle's reduction. The counter all-reduce itself runs in
real processes (gloo, world size 2) on real decode outputs."""
import json
import os
import socket

import numpy as np
import pytest

from tests.conftest import GOLDEN
from qkd_ldpc_amd.dist import shard_range

FIX = os.path.join(GOLDEN, "config4_1m.npz")
WORLD = 8


@pytest.fixture(scope="module")
def c4():
    z = np.load(FIX)
    f = z["iters"].size
    return {"iters": z["iters"], "sp": np.unpackbits(z["sp"])[:f].astype(bool),
            "ko": np.unpackbits(z["ko"])[:f].astype(bool), "q": float(z["exact_q"][0]),
            "stats": json.loads(str(z["stats"])), "frames": f}


def counters_of(iters, sp, ko):
    """qkd_counters bytes as counters_kernel writes them (include/qkd_ldpc.h)."""
    it = iters[sp].astype(np.uint64)
    rec = np.zeros(48, np.uint8)
    rec[:40] = np.array([len(iters), sp.sum(), (sp & ko).sum(), it.sum(), (it * it).sum()],
                        np.uint64).view(np.uint8)
    rec[40:48] = np.array([it.min() if it.size else 0xFFFFFFFF, it.max() if it.size else 0],
                          np.uint32).view(np.uint8)
    return rec


def reduce_records(recs):
    """SUM of the five uint64 sums, MIN / MAX of the extrema (dist.allreduce_counters)."""
    s = sum(r[:40].view(np.uint64) for r in recs)
    mn = min(int(r[40:44].view(np.uint32)[0]) for r in recs)
    mx = max(int(r[44:48].view(np.uint32)[0]) for r in recs)
    out = np.zeros(48, np.uint8)
    out[:40] = s.astype(np.uint64).view(np.uint8)
    out[40:48] = np.array([mn, mx], np.uint32).view(np.uint8)
    return out


def test_fixture_matches_its_own_aggregate(c4, oracle_mod):
    st = oracle_mod.batch_stats(c4["iters"], c4["sp"], c4["ko"], np.array([c4["q"]]), c4["frames"], 50)
    for k in ("iterations_successful_sp_mean", "iterations_successful_sp_std_dev", "fer",
              "iterations_successful_sp_min", "iterations_successful_sp_max", "sum_iters_sp"):
        assert st[k] == c4["stats"][k], k
    # config 2 is the first 4096 frames of config 4 (same seeds, same point)
    assert int(c4["iters"][:4096].astype(np.int64).sum()) == 12905
    assert c4["q"] == 204 / 10240


def test_oracle_prefix_matches_fixture(c4, oracle_code, oracle_mod):
    """A spot re-run of the oracle on frames inside every 125k shard."""
    seeds = oracle_mod.seeds(777, c4["frames"])
    for r in range(WORLD):
        b, e = shard_range(r, WORLD, c4["frames"])
        idx = np.arange(e - 64, e)
        got = oracle_code.trials(0.02, seeds[idx], 0, 50, 100.0, True, threads=8)
        assert (got["iters"] == c4["iters"][idx]).all()
        assert (got["sp_ok"] == c4["sp"][idx]).all() and (got["key_ok"] == c4["ko"][idx]).all()


def _worker(rank, world, port, iters, sp, ko, out):
    import torch
    import torch.distributed as dist
    from qkd_ldpc_amd.dist import allreduce_counters
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


def test_allreduce_of_real_shards_equals_whole_run(c4):
    """gloo world size 2 over the reference decode outputs of all 1M frames."""
    import torch.multiprocessing as mp
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(2, _free_port(), c4["iters"], c4["sp"], c4["ko"], out), nprocs=2, join=True)
    want = counters_of(c4["iters"], c4["sp"], c4["ko"]).tobytes()
    assert out[0] == want and out[1] == want


@pytest.mark.gpu
def test_config4_eight_shards_on_one_gpu(c4, oracle_mod):
    import torch
    import qkd_ldpc_amd as Q
    from tests.conftest import GOLDEN as G
    g = dict(np.load(os.path.join(G, "code_n10240.npz")))
    H = Q.HMatrix.from_check_lists(10240, g["chk_off"], g["chk_idx"])
    ws = Q.Workspace(H)
    F = c4["frames"]
    seeds_all = torch.from_numpy(Q.make_seeds(777, F).view(np.int64)).cuda()
    recs = []
    for r in range(WORLD):
        b, e = shard_range(r, WORLD, F)
        res = Q.run_trials(H, seeds_all[b:e].contiguous(), 0.02, 0, 50, 100.0, True, workspace=ws)
        torch.cuda.synchronize()
        it = res.iterations.cpu().numpy()
        bad = np.nonzero(it != c4["iters"][b:e])[0]
        assert bad.size == 0, f"shard {r}: {bad.size} frames differ, first {b + bad[:5]}"
        assert (res.syndromes_match.cpu().numpy().astype(bool) == c4["sp"][b:e]).all()
        assert (res.keys_match.cpu().numpy().astype(bool) == c4["ko"][b:e]).all()
        assert (res.exact_qber.cpu().numpy() == c4["q"]).all()
        rec = res.counters.cpu().numpy()
        assert rec.tobytes() == counters_of(c4["iters"][b:e], c4["sp"][b:e], c4["ko"][b:e]).tobytes()
        recs.append(rec)
        del res
    whole = Q.run_trials(H, seeds_all, 0.02, 0, 50, 100.0, True, workspace=ws)
    torch.cuda.synchronize()
    rec_whole = whole.counters.cpu().numpy()
    assert reduce_records(recs).tobytes() == rec_whole.tobytes()
    assert (whole.iterations.cpu().numpy() == c4["iters"]).all()
    st = Q.counters_to_stats(Q.read_counters(whole.counters), F, 50, c4["q"])
    for k in ("fer", "iterations_successful_sp_min", "iterations_successful_sp_max", "sum_iters_sp"):
        assert st[k] == c4["stats"][k], k
    # mean / std from exact integer sums agree with the reference's two-pass doubles to
    # the 6 significant digits its CSV prints (simulation.cpp:285-312, :26-35)
    for k in ("iterations_successful_sp_mean", "iterations_successful_sp_std_dev"):
        assert float(f"{st[k]:.6g}") == float(f"{c4['stats'][k]:.6g}"), k
