"""The multi-GPU path on the MI355X: RCCL itself (a world-size-1 "nccl" process
group all-reducing real counter records, the collective bench.py issues per step)
and `bench.py --gpus 2` starting its own ranks (gloo sharing the one device: RCCL
needs one GPU per rank). Replaces the reference's thread-pool fan-out of a point's
trials (simulation.cpp:230-250)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_rccl_allreduce_of_real_counters(tmp_path):
    from qkd_ldpc_amd.dist import spawn_ranks
    out = str(tmp_path / "nccl.json")
    rc = spawn_ranks(1, [os.path.join(ROOT, "tests", "dist_gpu_rank.py"), out])
    assert rc == 0
    res = json.load(open(out))
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["same_ok"], "a one-rank all-reduce must leave the counters unchanged"
    assert res["same_failed"] and res["failed_minmax"] == [0xFFFFFFFF, 0]
    c = np.array(res["counters"], np.uint8)
    sums = c[:40].view(np.uint64)
    assert sums[0] == 512 and sums[1] == 512 and sums[2] == 512


def test_bench_starts_its_own_ranks(golden_vectors):
    """`python bench.py --gpus 2` (no torchrun): two ranks on the one MI355X over gloo,
    each decoding its 512-frame share of the seed stream; the reduced counters are the
    golden per-frame outcomes of frames 0..1023."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["QKD_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--frames", "512", "--no-e2e", "--no-variants", "--no-cpu-baseline",
                        "--no-sweeps"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, p.stdout
    out = json.loads(line[0])
    assert out["n_gpus"] == 2
    it = golden_vectors["c2_iters"][:1024].astype(np.int64)
    sp = golden_vectors["c2_sp"][:1024].astype(bool)
    assert out["sum_iterations"] == int(it[sp].sum())
    assert out["fer"] == 0.0
    assert abs(out["value"] - 2 * 512 * 10240 * 2 / (out["ms_per_step"] * 2 / 1e3)) / out["value"] < 1e-6


def test_bench_config4_over_two_ranks():
    """BASELINE configs[3] through `python bench.py --gpus 2` (two ranks on the one
    MI355X over gloo): each rank runs its shard of the first 20,000 config-4 frames in
    one qkd_trials_batch, the counters are all-reduced, and the `config4` block's
    aggregate equals the oracle fixture's (tests/golden/config4_1m.npz) exactly."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["QKD_DIST_BACKEND"] = "gloo"
    frames = 20000
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--prewarm-ms", "0", "--frames", "256", "--no-e2e", "--no-variants",
                        "--no-cpu-baseline", "--config4-frames", str(frames)],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, p.stdout
    c4 = json.loads(line[0])["config4"]
    assert c4["n_gpus"] == 2 and c4["frames"] == frames and c4["frames_per_rank"] == frames // 2
    assert c4["matches_fixture"] is True, c4["counters"]
    assert c4["counters"]["frames"] == frames and c4["fer"] == 0.0
    assert abs(c4["value"] - frames * 10240 / (c4["ms"] / 1e3)) / c4["value"] < 1e-9


def test_counters_merge_kernel_matches_host_form():
    """qkd_counters_merge (the device half of dist.allreduce_counters: one launch after
    the all-gather) against the host form on eight records, one of them all-failed
    (UINT32_MAX / 0 extrema), the output aliasing the first record."""
    import torch
    from qkd_ldpc_amd.dist import merge_counters
    from test_dist import counters_of
    rng = np.random.default_rng(11)
    rows = []
    for k in range(8):
        f = 100 + 7 * k
        it = rng.integers(1, 51, f).astype(np.uint32)
        sp = (rng.random(f) < (0.0 if k == 5 else 0.8)).astype(np.uint8)
        ko = (rng.random(f) < 0.9).astype(np.uint8)
        rows.append(counters_of(it, sp, ko))
    host = torch.from_numpy(np.stack(rows))
    want = torch.empty(48, dtype=torch.uint8)
    merge_counters(host, want)
    dev = host.cuda()
    merge_counters(dev, dev[0])
    torch.cuda.synchronize()
    assert dev[0].cpu().numpy().tobytes() == want.numpy().tobytes()
