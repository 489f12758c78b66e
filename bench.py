"""Headline benchmark: decoded key bits/s of the N=10240 R=0.49 code at QBER 0.02,
<= 50 sum-product iterations, message clamp 100 (BASELINE.json configs[1]).

One step = one QBER-point batch of F=4096 frames through the hot path, keys
already resident in HBM: LLR init, Alice's syndrome, flooding sum-product
decode, key comparison and the batch counters (qkd_qkd_ldpc_batch +
qkd_counters_batch). Key pairs are generated once on the device beforehand
with the reference's seeding (SIMULATION_SEED=777, frame k -> seeds[k]).

Multi-GPU (torchrun, one process per GPU): frames shard with no data-path
collective; rank r decodes frames [r*F, (r+1)*F) of the seed stream (weak
scaling) and the counters are summed with one all-reduce per step.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_BITS = 10240
# Algorithmic bytes: reference two-array flooding formulation
# with binary64 messages. Per executed iteration: read+write b2c, read+write c2b
# (4 E w) plus the LLR read (N w); per frame: Bob's bits in, decoded bits out,
# syndrome in (2N + M bytes).
E_EDGES, M_CHECKS, W = 30720, 5231, 8
B_ITER = 4 * E_EDGES * W + N_BITS * W          # 1,064,960 (binary64 messages)
B_ITER32 = 4 * E_EDGES * 4 + N_BITS * 4        # 532,480 (binary32 variants)
B_FRAME = 2 * N_BITS + M_CHECKS                 # 25,711
HBM_PEAK_GBS = 8000.0                           # MI355X_MICROARCH.md, HBM3E spec


# decoder rules measured (include/qkd_ldpc.h QKD_VARIANT_*): the reference's,
# and the build-defined binary32 variants; minsum_sc = self-corrected min-sum at
# its best scale (profiles/r02_minsum_sweep.jsonl)
VARIANTS = {"sp_f64": {"variant": "sp_f64"}, "sp_f32": {"variant": "sp_f32"}, "minsum": {"variant": "minsum"},
            "minsum_sc": {"variant": "minsum", "minsum_scale": 0.875, "minsum_self_correct": True}}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under torchrun, else 1); without "
                         "torchrun, N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--prewarm-ms", type=float, default=250.0,
                    help="untimed steps before the W warmup steps until this much wall time has "
                         "passed (the GPU clock's ramp; 0 disables)")
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--qber", type=float, default=0.02)
    ap.add_argument("--max-iters", type=int, default=50)
    ap.add_argument("--threshold", type=float, default=100.0)
    ap.add_argument("--seed", type=int, default=777)
    ap.add_argument("--cpu-frames", type=int, default=8192,
                    help="frames in the CPU-baseline sample (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="CPU-baseline threads (capped at the CPUs this process may use)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (keygen + decode) line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--variant", default="sp_f64", choices=sorted(VARIANTS),
                    help="decoder rule of the headline line (sp_f64 = the reference's)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the side measurement of the binary32 variants")
    ap.add_argument("--kernel-events", choices=["on", "off"], default="on",
                    help="HIP events around each decoder launch inside the timed loop (off: diagnostics)")
    ap.add_argument("--no-sweeps", action="store_true",
                    help="skip the config-3 QBER sweep (and config 4, as --config4-frames 0)")
    ap.add_argument("--config4-frames", type=int, default=None,
                    help="frames of the configs[3] run sharded over the ranks (default 1,000,000, "
                         "0 with --no-sweeps; 0 disables)")
    ap.add_argument("--phase-timing", action="store_true",
                    help="per-phase shader-clock shares of the decoder (diagnostic; the QKD_PHASE_TIMING "
                         "option)")
    ap.add_argument("--debug-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a library debug / A-B option (qkd_debug_set_option, include/qkd_ldpc.h), "
                         "process-wide; repeatable. The library reads no environment variable")
    args = ap.parse_args()
    if args.config4_frames is None:
        args.config4_frames = 0 if args.no_sweeps else 1_000_000
    return args


def load_code(device):
    import qkd_ldpc_amd as Q
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz")))
    return Q.HMatrix.from_check_lists(int(g["dims"][0]), g["chk_off"], g["chk_idx"],
                                      device=device), g


# The oracle (oracle/oracle.c) against the reference on the same 8-core Xeon of the
# build container, config 2 (4096 frames): the reference's 2.66-2.76 s were measured
# by the survey; the oracle's time is tools/cpu_calibrate.py's.
REF_C2_8T_S = (2.66, 2.76)
ORACLE_C2_8T_S = None      # filled in from profiles/cpu_calibration.json when present


def pmc_record(variant):
    """Per-launch PMC record of the variant's decode kernel (newest
    profiles/r*_pmc_<variant>.json, written by tools/pmc_traffic.py from separate
    rocprofv3 --pmc passes, gfx950 FETCH_SIZE x2)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{variant}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], ROOT)


def rocprof_warm_ms(kernel):
    """Warm average duration of `kernel` in the newest committed rocprofv3
    --kernel-trace summary (profiles/r*_kernel_summary.json, tools/prof_summary.py)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_summary.json")))
    for path in reversed(files):
        with open(path) as f:
            for r in json.load(f)["kernels"]:
                if r["kernel"] == kernel:
                    return r["warm_avg_ms"], os.path.relpath(path, ROOT)
    return None, None


N_SIMD = 1024            # 256 CUs x 4 SIMD-32 units
VALU_ISSUE_CYC = 2.0     # cycles per wave64 VALU instruction on a SIMD-32 (MI355X_MICROARCH.md)
RATED_CLOCK_GHZ = 2.4    # MI355X peak engine clock


def issue_ceiling_4waves():
    """Cycles per wave-instruction per SIMD that 4 waves per SIMD (this decoder's
    occupancy: one 1024-thread workgroup per CU) sustain at ILP 8, by instruction kind,
    from the newest committed tools/mb/issue_mb.hip record (profiles/r*_issue_mb.txt)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_issue_mb.txt")))
    if not files:
        return None
    out = {}
    with open(files[-1]) as f:
        for line in f:
            p = line.split()
            # "<inst> waves/SIMD <w> ILP <k> cycles/wave-inst/SIMD <c>"
            if len(p) == 7 and p[1] == "waves/SIMD" and float(p[2]) == 4.0 and p[4] == "8":
                out[p[0]] = float(p[6])
    return {"cycles_per_wave_inst": out, "source": os.path.relpath(files[-1], ROOT)} if out else None


def roofline_block(variant, alg_bytes, kernel_s, call_s, kernel_name):
    """roofline (the contract's block) for the decode kernel, bound by what binds it.

    The decoder is VALU-issue / latency bound, not HBM bound: its
    speculative rounds run binary32 intervals and most message slots sit in LDS, so it
    never moves the reference's two-array binary64 bytes. The headline is therefore
    the VALU issue fraction of the kernel's PMC record (separate rocprofv3 --pmc
    passes, tools/pmc_traffic.py), priced by instruction mix and reproducible from
    that file, profiles/r*_valu_census.json and profiles/r*_issue_mb.txt alone:
        frac = sum over VALU classes (SQ_INSTS_VALU_<class> x its 4-wave issue cost)
               / (kernel cycles x 1024 SIMDs)
    with kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs of the counted dispatches, and a
    class's cost the mean of its opcodes' costs measured at this decoder's occupancy
    (4 waves per SIMD, tools/mb/issue_mb.hip), weighted by the kernel's dynamic opcode
    census (tools/valu_census.py) -- the unclassified rest (selects, moves, shifts,
    compares, lane reads) included;
    achieved = the needed SIMD-issue cycles per second and peak = 1024 SIMDs x the
    effective clock, so frac = achieved / peak. frac_2cyc keeps every instruction at
    2 cycles (SQ_INSTS_VALU x 2 / (kernel cycles x 1024), a lower bound of the issue
    time). A record without the class counters falls back to frac_2cyc.
    Beside it:
      live              the same instruction count over THIS run's decoder time (HIP
                        events around each launch on its stream), at the PMC pass's
                        effective clock and at the rated 2.4 GHz;
      hbm_frac_measured the PMC record's HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) per
                        launch over the counted dispatches' duration, / 8 TB/s;
      nominal_frac      SURVEY.md §8(d)'s algorithmic bytes (the reference's two-array
                        binary64 traffic at the executed iterations) over the live kernel
                        time / 8 TB/s -- above 1 when the kernel finishes sooner than any
                        HBM-bound implementation of that formulation could: it is NOT an
                        achieved bandwidth;
      issue_ceiling_4waves  what 4 waves per SIMD sustain per instruction kind
                        (tools/mb/issue_mb.hip), a second reference point."""
    rec, src = pmc_record(variant)
    nominal = alg_bytes / kernel_s / 1e9 / HBM_PEAK_GBS
    base = {"kernel": kernel_name, "kernel_ms": kernel_s * 1e3, "call_ms": call_s * 1e3,
            "algorithmic_bytes_per_launch": alg_bytes, "nominal_frac": nominal,
            "nominal_note": "SURVEY.md §8(d) bytes / live kernel time / 8 TB/s; exceeds 1 because this kernel "
                            "does not move the reference's two-array fp64 bytes -- not an achieved bandwidth",
            "nominal_frac_call": alg_bytes / call_s / 1e9 / HBM_PEAK_GBS}
    v = (rec or {}).get("valu", {})
    insts, cyc, clk = v.get("valu_insts_per_launch"), v.get("gpu_cycles"), v.get("effective_clock_ghz")
    if not (rec and insts and cyc and clk):
        # no PMC record: only the nominal HBM figure is available (marked so)
        return {"bound": "hbm", "achieved": alg_bytes / kernel_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": nominal, "traffic": None, "nominal": True, **base}
    pmc_s = cyc / (clk * 1e9)                        # the counted dispatches' duration
    frac_2cyc = insts * VALU_ISSUE_CYC / (cyc * N_SIMD)
    # the record's VALU classes priced now, from the committed opcode census and
    # issue table (tools/pmc_traffic.py valu_mix; a record without the class
    # counters keeps frac_2cyc)
    mix = None
    if "SQ_INSTS_VALU_FMA_F32" in rec.get("counters", {}):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import pmc_traffic
        # (a binary32 variant: its own kernel's census, tools/valu_census.py variant)
        cpath = None if variant == "sp_f64" else pmc_traffic.newest(f"r*_valu_census_{variant}.json")
        mix = pmc_traffic.valu_mix(rec["counters"], cyc, census_path=cpath)
    if mix:
        # the kernel's own VALU instruction mix priced at what 4 waves per SIMD
        # issue (tools/pmc_traffic.py valu_mix): achieved = SIMD-cycles of VALU
        # issue the launch needs per second, peak = 1024 SIMDs x the clock
        achieved = mix["simd_cycles_needed"] / pmc_s / 1e9
        peak = N_SIMD * clk
        out = {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "G SIMD-issue-cycles/s",
               "frac": mix["frac_mix"], "frac_2cyc": frac_2cyc,
               "formula": "frac = sum over VALU classes (PMC count x the census-weighted 4-wave issue cost of "
                          "the class's opcodes) / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); frac_2cyc = SQ_INSTS_VALU x 2 "
                          "/ (GRBM_GUI_ACTIVE/8 x 1024), every instruction at 2 cycles",
               "mix": mix}
    else:
        out = {"bound": "valu", "achieved": insts / pmc_s / 1e9, "peak": N_SIMD / VALU_ISSUE_CYC * clk,
               "unit": "G wave-inst/s", "frac": frac_2cyc, "frac_2cyc": frac_2cyc,
               "formula": "frac = SQ_INSTS_VALU x 2 / (GRBM_GUI_ACTIVE/8 x 1024) of the PMC record"}
    out.update({"traffic": rec.get("hbm_bytes_per_launch"),
           "pmc_source": src, "pmc_kernel": rec.get("kernel"),
           "valu_insts_per_launch": insts, "pmc_kernel_cycles": cyc, "pmc_clock_ghz": clk,
           "pmc_kernel_ms": pmc_s * 1e3,
           "hbm_frac_measured": rec["hbm_bytes_per_launch"] / pmc_s / 1e9 / HBM_PEAK_GBS,
           "live": {"kernel_ms": kernel_s * 1e3,
                    "frac_at_pmc_clock": insts * VALU_ISSUE_CYC / (kernel_s * clk * 1e9 * N_SIMD),
                    "frac_at_rated_clock": insts * VALU_ISSUE_CYC / (kernel_s * RATED_CLOCK_GHZ * 1e9 * N_SIMD),
                    "frac_mix_at_pmc_clock": (mix["simd_cycles_needed"] / (kernel_s * clk * 1e9 * N_SIMD)
                                              if mix else None)},
           "valu_active_frac": v.get("valu_active_util_x4"), "wait_frac": v.get("wait_frac"),
           "lds_conflict_frac": v.get("lds_conflict_frac"), **base})
    ceil = issue_ceiling_4waves()
    if ceil:
        c = ceil["cycles_per_wave_inst"]
        out["issue_ceiling_4waves"] = ceil
        if "v_fma_f32" in c:
            out["frac_of_4wave_fma_ceiling"] = insts * c["v_fma_f32"] / (cyc * N_SIMD)
    warm, wsrc = rocprof_warm_ms(rec.get("kernel"))
    if warm:
        out["rocprof_warm_ms"] = warm
        out["rocprof_source"] = wsrc
    return out


def decoder_ms(L, ws, start):
    """qkd_debug_decoder_timing: start, or collect the average decoder-kernel ms."""
    import ctypes as C
    from qkd_ldpc_amd import _native as N
    tot, n = C.c_double(0), C.c_uint64(0)
    N.check(L.qkd_debug_decoder_timing(ws.handle, 1 if start else 0, C.byref(tot), C.byref(n)))
    return tot.value / n.value if n.value else None


def measure_variants(args, step, stream, counters, iters, Q, F, q, L, ws, steps=5):
    """Side measurement on the same resident keys: the build-defined binary32
    variants (QKD_VARIANT_SP_F32, QKD_VARIANT_MINSUM plain and self-corrected;
    SURVEY.md §8(d) config 5),
    timed like the headline (wall clock over `steps` steps, HIP events around the
    decode kernel and around the call). Their FER is a property of the decoder, not a
    parity claim. Their roofline block's `bound` is what their PMC record shows (their
    message stores live in LDS: they are not HBM-bound)."""
    import torch
    out = {}
    for v in VARIANTS:
        if v == args.variant:
            continue
        step(variant=v)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(steps)]
        decoder_ms(L, ws, True)
        t0 = time.perf_counter()
        for k in range(steps):
            step(evs[k], variant=v)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kms = decoder_ms(L, ws, False)
        st = Q.counters_to_stats(Q.read_counters(counters), F, args.max_iters, q)
        cms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        b_iter = B_ITER if v == "sp_f64" else B_ITER32
        alg = int(iters.cpu().numpy().astype(np.int64).sum()) * b_iter + F * B_FRAME
        rb = roofline_block(v, alg, kms / 1e3, cms / 1e3, f"decoder kernel of qkd_qkd_ldpc_batch, variant {v}")
        out[v] = {"value": F * N_BITS * steps / el, "unit": "bit/s", "kernel_ms": kms, "call_ms": cms,
                  "fer": st["fer"], "mean_iterations": st["iterations_successful_sp_mean"], "roofline": rb}
    return out


def measure_end_to_end(args, H, ws, seeds, F, Q, steps):
    """End to end per SURVEY.md §8(d) / run_trial (simulation.cpp:161-189): device
    keygen + LLR + syndrome + decode + key compare + counters, one qkd_trials_batch
    per step from the seeds alone."""
    import torch
    res = Q.run_trials(H, seeds, args.qber, 0, args.max_iters, args.threshold, True, workspace=ws)
    torch.cuda.synchronize()
    # untimed calls for --prewarm-ms first, as before the decode-only steps: the
    # GPU idles while the host prepares this measurement, and its clock takes
    # ~0.2 s of work to return (a kernel trace of the first end-to-end steps:
    # the decoder 1.27 -> 1.38 -> ... 1.19 ms over ~20 steps)
    t_pw = time.perf_counter()
    while (time.perf_counter() - t_pw) * 1e3 < args.prewarm_ms:
        for _ in range(5):
            Q.run_trials(H, seeds, args.qber, 0, args.max_iters, args.threshold, True, workspace=ws, out=res)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        Q.run_trials(H, seeds, args.qber, 0, args.max_iters, args.threshold, True, workspace=ws, out=res)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = Q.counters_to_stats(Q.read_counters(res.counters), F, args.max_iters,
                             float(res.exact_qber[0].item()))
    return {"value": F * N_BITS * steps / el, "unit": "bit/s", "ms_per_step": el * 1e3 / steps,
            "steps": steps, "fer": st["fer"], "sum_iterations": st["sum_iters_sp"],
            "what": "qkd_trials_batch: keygen_split_kernel + frame_syn + decoder (key compare in its epilogue) + counters"}


def config3_sweep(args, H, Q, dev):
    """BASELINE configs[2]: the FER curve, QBER 0.01 ... 0.08 (qber_range(0.01, 0.09, 0.01)),
    10,000 trials per point, point s seeding frame k with seeds[k] + s
    (simulation.cpp:231-312), one qkd_trials_batch per point (device keygen included,
    as run_trial times it) on a fresh workspace, in the reference's point order. The
    reference's own table (measured on 8 Xeon threads in 145.5 s) sits
    beside each point; with the bit-exact decoder FER and mean iterations must equal it
    to its printed digits."""
    import torch
    with open(os.path.join(ROOT, "tests", "golden", "reference_probe.json")) as f:
        ref = json.load(f)["config3"]
    trials = ref["trials"]
    grid = Q.qber_range(ref["qber_begin"], ref["qber_end"], ref["qber_step"])
    seeds = torch.from_numpy(Q.make_seeds(args.seed, trials).view(np.int64)).to(dev)
    ws = Q.Workspace(H)
    Q.run_trials(H, seeds[:256], grid[0], 0, args.max_iters, args.threshold, True, workspace=ws)   # warm
    torch.cuda.synchronize()
    points, total = [], 0.0
    for s_, qn in enumerate(grid):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = Q.run_trials(H, seeds, qn, s_, args.max_iters, args.threshold, True, workspace=ws)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        total += dt
        st = Q.counters_to_stats(Q.read_counters(r.counters), trials, args.max_iters,
                                 float(r.exact_qber[0].item()))
        rp = ref["points"][s_]
        points.append({"qber_nominal": qn, "qber_actual": float(r.exact_qber[0].item()), "ms": dt * 1e3, "fer": st["fer"],
                       "mean_iterations": st["iterations_successful_sp_mean"],
                       "sum_iterations": st["sum_iters_sp"],
                       "reference": {"qber_actual": rp["qber_actual"], "fer": rp["fer"], "mean_it": rp["mean_it"]},
                       "matches_reference": bool(abs(st["fer"] - rp["fer"]) < 1e-12 and
                                                 abs(st["iterations_successful_sp_mean"] - rp["mean_it"])
                                                 <= 5e-4 + 1e-9)})
    ws.close()
    return {"what": "configs[2]: 8 QBER points x 10,000 trials, qkd_trials_batch per point (keygen + decode + "
                    "counters), fresh workspace, ascending points", "total_s": total,
            "reference_total_s_8_xeon_threads": 145.5, "points": points}


def config4_fixture_counters(frames):
    """The qkd_counters record (include/qkd_ldpc.h) of config-4 frames [0, frames)
    from the oracle's per-frame fixture tests/golden/config4_1m.npz, or None when the
    run is longer than the fixture."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "config4_1m.npz"))
    n = z["iters"].size
    if frames > n:
        return None
    sp = np.unpackbits(z["sp"])[:frames].astype(bool)
    ko = np.unpackbits(z["ko"])[:frames].astype(bool)
    it = z["iters"][:frames][sp].astype(np.uint64)
    return {"frames": frames, "sp_ok": int(sp.sum()), "ldpc_ok": int((sp & ko).sum()),
            "sum_iters": int(it.sum()), "sum_iters_sq": int((it * it).sum()),
            "min_iters": int(it.min()) if it.size else 0xFFFFFFFF, "max_iters": int(it.max()) if it.size else 0}


def config4(args, H, Q, dev, rank, world):
    """BASELINE configs[3]: the config-2 point with --config4-frames (1,000,000) frames
    sharded over the ranks (the reference's thread-pool fan-out
    simulation.cpp:230-250 and its reduction :252-312). Rank r takes
    shard_range(r, world, F) of the one seed stream, runs ONE qkd_trials_batch (device
    keygen + frame syndromes + decode + key compare + counters), and the counters are
    all-reduced (RCCL under torchrun / --gpus N). Timed between a barrier +
    synchronize on both sides, max over ranks; an untimed run of the same shard first
    (workspace allocation, clocks). value = F * N bits / that time."""
    import torch
    from qkd_ldpc_amd.dist import imbalance, run_sharded_point
    F = args.config4_frames
    ws = Q.Workspace(H)
    res = {}

    def run_shard(b, e):
        if "r" not in res:
            res["seeds"] = torch.from_numpy(Q.make_seeds(args.seed, e)[b:e].view(np.int64)).to(dev)
            res["r"] = Q.run_trials(H, res["seeds"], args.qber, 0, args.max_iters, args.threshold, True,
                                    workspace=ws)
        else:
            Q.run_trials(H, res["seeds"], args.qber, 0, args.max_iters, args.threshold, True, workspace=ws,
                         out=res["r"])
        return res["r"].counters

    counters, dt, (b, e), per_rank = run_sharded_point(rank, world, F, run_shard, torch.cuda.synchronize)
    c = Q.read_counters(counters)
    q = float(res["r"].exact_qber[0].item())
    ws.close()
    got = {"frames": int(c.frames), "sp_ok": int(c.sp_ok), "ldpc_ok": int(c.ldpc_ok),
           "sum_iters": int(c.sum_iters), "sum_iters_sq": int(c.sum_iters_sq),
           "min_iters": int(c.min_iters), "max_iters": int(c.max_iters)}
    want = config4_fixture_counters(F)
    st = Q.counters_to_stats(c, F, args.max_iters, q)
    return {"what": f"configs[3]: {F} config-2 frames over {world} rank(s), one qkd_trials_batch per rank "
                    "(keygen + decode + counters), counters all-reduced, max-rank time",
            "frames": F, "n_gpus": world, "frames_per_rank": e - b, "ms": dt * 1e3,
            "per_rank_ms": [t * 1e3 for t in per_rank], "imbalance_max_over_min": imbalance(per_rank),
            "value": F * N_BITS / dt, "unit": "bit/s", "fer": st["fer"],
            "sum_iterations": got["sum_iters"], "mean_iterations": st["iterations_successful_sp_mean"],
            "std_iterations": st["iterations_successful_sp_std_dev"], "counters": got,
            "matches_fixture": (got == want) if want is not None else None,
            "fixture": "tests/golden/config4_1m.npz (oracle per-frame results, frames [0, F))"}


def cpu_calibration():
    p = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    ref = sum(REF_C2_8T_S) / 2
    return {"oracle_c2_8threads_s": d["oracle_c2_seconds"], "reference_c2_8threads_s": list(REF_C2_8T_S),
            "oracle_over_reference_time": d["oracle_c2_seconds"] / ref,
            "where": d.get("host", "build container, 8-core Xeon"), "source": "profiles/cpu_calibration.json"}


def cpu_baseline(args, g):
    """The oracle (CPU restatement of the reference, glibc libm, -O3) on a bounded
    sample of the same workload, one frame per task on `threads` host threads.

    Core count: the GPU box gives each GPU a 16-CPU host share (worker pools are
    sized to it there: OMP_NUM_THREADS and the pool's rules), while
    os.sched_getaffinity shows the whole machine. The measured figure uses that
    share (`cores`); `all_cores_estimate` scales it linearly to every affinity CPU
    (the reference's frames are independent tasks on a thread pool,
    simulation.cpp:230-250, so its throughput scales with cores until memory
    bandwidth binds: an upper estimate, not a measurement)."""
    from oracle import oracle as O
    O.build()
    code = O.Code.from_lists(g)
    frames = args.cpu_frames
    seeds = O.seeds(args.seed, frames)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    threads = max(1, min(args.cpu_threads, avail))
    t0 = time.perf_counter()
    r = code.trials(args.qber, seeds, 0, args.max_iters, args.threshold, True, threads=threads)
    dt = time.perf_counter() - t0
    cal = cpu_calibration()
    value = frames * N_BITS / dt
    ratio = cal["oracle_over_reference_time"] if cal else None
    return {
        "value": value,
        "unit": "bit/s",
        "reference_equivalent_value": value * ratio if cal else None,
        "cores": threads,
        "kind": "port",
        "sample": f"{frames} frames of the same config (seeds 777[0:{frames}]), "
                  f"{threads} threads, {dt:.2f} s wall, mean it "
                  f"{float(np.mean(r['iters'])):.4f}",
        "host_cpus_visible": os.cpu_count(),
        "host_cpus_affinity": avail,
        "all_cores_estimate": {"cores": avail, "value": value * avail / threads,
                               "reference_equivalent_value": value * avail / threads * ratio if cal else None,
                               "how": f"linear scaling of the {threads}-thread measurement to {avail} CPUs "
                                      "(not run: the box's worker-pool share is 16 CPUs per GPU)"},
        "cores_note": "one thread per core of this GPU's host CPU share (16 per GPU on the "
                      "MI355X pool; os.cpu_count() shows the whole machine)",
        "calibration": cal,
    }


def main():
    args = parse()
    from qkd_ldpc_amd.dist import init_rank, rank_env, spawn_ranks

    env = rank_env()
    if env is None and (args.gpus or 1) > 1:
        # one process per GPU, started here (no HIP call in this parent process)
        sys.exit(spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    rank, world, local = env or (0, 1, 0)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with the launcher's WORLD_SIZE {world}")
    import torch
    import torch.distributed as dist

    if env is not None:
        # RCCL ("nccl") with one device per rank; QKD_DIST_BACKEND=gloo with more
        # ranks than GPUs rehearses the multi-rank path on one device (tests)
        init_rank(world, local)
    import qkd_ldpc_amd as Q

    for kv in args.debug_opt + (["QKD_PHASE_TIMING=1"] if args.phase_timing else []):
        name, _, value = kv.partition("=")
        Q.set_debug_option(name, value)
    H, g = load_code(torch.cuda.current_device())
    dev = torch.device("cuda", torch.cuda.current_device())
    from qkd_ldpc_amd.dist import allreduce_counters, imbalance, rank_times, shard_range
    F = args.frames
    all_seeds = Q.make_seeds(args.seed, F * world)
    b, e = shard_range(rank, world, F * world)          # weak scaling: F frames per rank
    seeds = torch.from_numpy(all_seeds[b:e].view(np.int64)).to(dev)
    ws = Q.Workspace(H)
    stream = torch.cuda.current_stream()

    # key pairs resident in HBM before the timed region
    alice, bob, exact_q = Q.keygen(H, seeds, args.qber, 0, workspace=ws)
    q = float(exact_q[0].item())
    iters = torch.empty(F, dtype=torch.int32, device=dev)
    sp = torch.empty(F, dtype=torch.uint8, device=dev)
    ko = torch.empty(F, dtype=torch.uint8, device=dev)
    counters = torch.empty(Q._native.COUNTERS_BYTES, dtype=torch.uint8, device=dev)
    L = Q._native.lib()
    sptr = int(stream.cuda_stream)

    def step(ev=None, variant=args.variant, reduce=True):
        flags = Q.decoder_flags(True, **VARIANTS[variant])
        if ev is not None:
            ev[0].record(stream)
        Q._native.check(L.qkd_qkd_ldpc_batch(H.handle, ws.handle, alice.data_ptr(), bob.data_ptr(), F,
                                             q, args.max_iters, args.threshold, flags,
                                             None, iters.data_ptr(), sp.data_ptr(), ko.data_ptr(), sptr))
        if ev is not None:
            ev[1].record(stream)
        Q._native.check(L.qkd_counters_batch(iters.data_ptr(), sp.data_ptr(), ko.data_ptr(), F,
                                             counters.data_ptr(), H.device, sptr))
        if world > 1 and reduce:
            allreduce_counters(counters)

    Q.spec_replays(ws, reset=True)
    # The GPU's clock ramps over its first ~40 ms of work (tools/warm_probe.py,
    # profiles/r03_warm_probe.txt: 1.83 -> 1.70 ms per step), longer than W
    # warmup steps of a 2 ms step take: untimed steps fill --prewarm-ms first,
    # so the K timed steps see steady-state clocks, as a QKD post-processing
    # pipeline running continuously does. Then the W warmup steps proper.
    # (Timed by each rank's own clock, so ranks run different numbers of
    # prewarm steps: those skip the counter all-reduce, which every rank must
    # enter equally often.)
    prewarm_steps = 0
    t_pw = time.perf_counter()
    while (time.perf_counter() - t_pw) * 1e3 < args.prewarm_ms:
        for _ in range(5):
            step(reduce=False)
        prewarm_steps += 5
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if args.kernel_events == "on":
        decoder_ms(L, ws, True)      # HIP events around each decoder launch, on its stream
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    torch.cuda.synchronize()
    own_elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if args.kernel_events == "on":
        dec_ms = decoder_ms(L, ws, False)
    else:
        decoder_ms(L, ws, True)
        for k in range(3):
            step()
        dec_ms = decoder_ms(L, ws, False)
    # every rank's own time, barrier-inclusive time and decoder-kernel time in one
    # all-gather: the max is the job's time, the spread its load imbalance
    per_rank = rank_times([own_elapsed, elapsed, dec_ms or 0.0], world)
    elapsed = max(r[1] for r in per_rank)
    # the whole library call (pack, frame syndromes, decoder), HIP events around it,
    # in a short untimed pass after the timed region
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for k in range(5):
        step(evs[k])
    torch.cuda.synchronize()
    kernel_ms = [a.elapsed_time(b) for a, b in evs]

    c = Q.read_counters(counters)
    it_np = iters.cpu().numpy()
    frames_total = F * world
    value = frames_total * N_BITS * args.steps / elapsed
    # per-launch algorithmic bytes on this rank (executed iterations)
    sum_it_local = int(it_np.astype(np.int64).sum())
    b_iter = B_ITER if args.variant == "sp_f64" else B_ITER32
    alg_bytes = sum_it_local * b_iter + F * B_FRAME
    avg_call_s = float(np.mean(kernel_ms)) / 1e3
    avg_kernel_s = dec_ms / 1e3
    replays = Q.spec_replays(ws, reset=True)

    stats = Q.counters_to_stats(c, frames_total, args.max_iters, q)
    if rank == 0:
        out = {
            "metric": "decoded key bits/sec + FER, N=10240 R=0.49 @ QBER=0.02, 50 iters",
            "value": value,
            "unit": "bit/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm": {"ms": args.prewarm_ms, "steps": prewarm_steps,
                        "note": "untimed steps before the warmup steps (GPU clock ramp, DESIGN.md §5)"},
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.variant == "sp_f64" else "f32",
            "data": "synthetic: reference keygen (xoshiro256++ seed 777, exact-QBER error "
                    "injection) on the device; reference alist code N=10240",
            "config": {
                "workload": "configs[1]: alist (N=10240,M=5231,R=0.49,CW=3,SEED=666), "
                            f"QBER {args.qber}, <= {args.max_iters} iterations, clamp "
                            f"{args.threshold}, {F}-frame batch per GPU",
                "frames_per_gpu": F,
                "decoder": args.variant,
                "parallelism": f"frames sharded over {world} GPU(s), counters all-reduced",
            },
            "fer": stats["fer"],
            "mean_iterations": stats["iterations_successful_sp_mean"],
            "sum_iterations": stats["sum_iters_sp"],
            "roofline": roofline_block(
                args.variant, alg_bytes, avg_kernel_s, avg_call_s,
                "decode_split_kernel (HIP events around its launch on its stream); call = "
                "qkd_qkd_ldpc_batch: pack + frame syndromes + decoder (key compare in its epilogue)"),
            "speculation": {
                "replayed_frames": replays,
                "frames": F * (prewarm_steps + args.warmup + args.steps + 5 + (3 if args.kernel_events == "off" else 0)),
                "note": "frames whose interval iterations could not certify every hard "
                        "decision, decoded again exactly (outputs bit-exact either way)",
            },
        }
        if world > 1:
            out["per_rank"] = {
                "step_ms": [r[0] * 1e3 / args.steps for r in per_rank],
                "decoder_kernel_ms": [r[2] for r in per_rank],
                "imbalance_step": imbalance([r[0] for r in per_rank]),
                "imbalance_decoder": imbalance([r[2] for r in per_rank]) if all(r[2] for r in per_rank) else None,
                "note": "each rank's own timed loop (before the closing barrier) and its mean decoder "
                        "kernel time (HIP events); imbalance = max / min",
            }
        if args.phase_timing:
            cyc = np.zeros(7, np.uint64)
            Q._native.check(L.qkd_debug_phase_cycles(ws.handle, cyc.ctypes.data))
            names = ["prologue", "check", "bit", "syndrome", "fetch_out", "check_first", "check_second"]
            tot = float(cyc.sum()) or 1.0
            out["phase_share"] = {n: float(v) / tot for n, v in zip(names, cyc)}
            out["phase_cycles"] = {n: int(v) for n, v in zip(names, cyc)}
        if world == 1 and not args.no_e2e:
            out["end_to_end"] = measure_end_to_end(args, H, ws, seeds, F, Q, args.steps)
        if world == 1 and not args.no_variants:
            out["variants"] = measure_variants(args, step, stream, counters, iters, Q, F, q, L, ws)
        if world == 1 and not args.no_sweeps:
            out["config3_sweep"] = config3_sweep(args, H, Q, dev)
    # BASELINE configs[3] on every rank (a collective: all ranks take part)
    c4 = config4(args, H, Q, dev, rank, world) if args.config4_frames > 0 else None
    if rank == 0:
        if c4 is not None:
            out["config4"] = c4
        if world == 1 and not args.no_cpu_baseline and args.cpu_frames > 0:
            out["cpu_baseline"] = cpu_baseline(args, g)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
