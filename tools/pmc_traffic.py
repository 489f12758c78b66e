"""Per-launch PMC record of the decode kernel from separate rocprofv3 --pmc passes
(tools/gpu_pmc.sh), corrected as /opt/skills/guides/MI355X_MICROARCH.md prescribes
for gfx950: FETCH_SIZE (KB) reports 1/2 of the bytes of wide reads -> x2; WRITE_SIZE
(KB) as is.

    python tools/pmc_traffic.py OUT.json SUMMARY.json DIR [DIR ...]

Every DIR holds one pass's run_counter_collection.csv. The decode kernel is the one
dispatch name containing "decode" (the bench runs one decoder variant per pass);
QKD_PMC_KERNEL overrides. SUMMARY.json is tools/prof_summary.py's output of the
kernel-trace pass: the kernel's warm average duration gives the effective clock.
"""
import collections
import csv
import json
import os
import sys

N_SIMD = 1024          # 256 CUs x 4 SIMDs
N_XCD = 8


def collect(dirs):
    """Counter values per kernel and counter, and per kernel and counter the
    dispatch durations (ns, End - Start of the same dispatch rows)."""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[r["Kernel_Name"]][r["Counter_Name"]].append(
                    float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return per, dur


# VALU issue cost per wave64 instruction per SIMD at 4 waves per SIMD (the split
# decoder's occupancy), ILP 8, shader cycles: tools/mb/issue_mb.hip,
# profiles/r05_issue_mb.txt. Packed binary32 ops count ONCE in the
# SQ_INSTS_VALU_{FMA,MUL,ADD}_F32 counters (the ISA census of the check-phase
# loops times their trip counts reproduces FMA_F32 to 2 %), so each class is
# priced at its packed share (same census) of the packed cost.
ISSUE_MB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "profiles", "r05_issue_mb.txt")


def issue_costs(path=ISSUE_MB, waves=4.0, ilp=8):
    """{instruction: cycles per wave-instruction per SIMD} at `waves` waves/SIMD and
    the given ILP, from the committed issue micro-benchmark output."""
    out = {}
    for line in open(path):
        f = line.split()
        if len(f) == 7 and float(f[2]) == waves and int(f[4]) == ilp:
            out[f[0]] = float(f[6])
    return out


# packed shares per class (census of the paired and iteration-2 check-phase steps
# and the speculative bit-phase rounds, weighted by their config-2 trip counts)
PACKED_SHARE = {"FMA_F32": 0.62, "MUL_F32": 0.45, "ADD_F32": 0.63}
OTHER_KINDS = ("v_mov_b32", "v_xor_b32", "v_bfe_u32", "v_med3_f32", "v_cmp_gt_f32", "v_cndmask_b32_sgpr")


def valu_mix(c, cycles):
    """The VALU instruction mix of the PMC record priced at the 4-wave issue
    costs: the SIMD-cycles the kernel's VALU stream needs at those rates, and the
    share of the kernel's SIMD-cycles that is (frac_mix = the issue-bound
    fraction at the kernel's own instruction mix)."""
    keys = ["SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32",
            "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32"]
    if not all(k in c for k in keys + ["SQ_INSTS_VALU"]) or not cycles:
        return None
    I = issue_costs()
    price = {
        "FMA_F32": PACKED_SHARE["FMA_F32"] * I["v_pk_fma_f32"] + (1 - PACKED_SHARE["FMA_F32"]) * I["v_fma_f32"],
        "MUL_F32": PACKED_SHARE["MUL_F32"] * I["v_pk_mul_f32"] + (1 - PACKED_SHARE["MUL_F32"]) * I["v_mul_f32"],
        "ADD_F32": PACKED_SHARE["ADD_F32"] * I["v_pk_add_f32"] + (1 - PACKED_SHARE["ADD_F32"]) * I["v_add_f32"],
        "TRANS_F32": (I["v_exp_f32"] + I["v_log_f32"] + I["v_rcp_f32"]) / 3,
        "F64": I["v_fma_f64"], "TRANS_F64": 2 * I["v_fma_f64"],
        "INT32": I["v_add_u32"], "INT64": 2 * I["v_add_u32"], "CVT": I["v_add_u32"],
        # the rest (selects, compares, moves, logic, med3 / max, lane reads): the
        # mean of the measured v_mov, v_xor, v_bfe, v_med3, v_cmp and v_cndmask
        # (SGPR mask, as compiled) costs
        "OTHER": sum(I[k] for k in OTHER_KINDS) / len(OTHER_KINDS),
    }
    g = lambda k: c.get("SQ_INSTS_VALU_" + k, 0.0)
    n = {"FMA_F32": g("FMA_F32"), "MUL_F32": g("MUL_F32"), "ADD_F32": g("ADD_F32"), "TRANS_F32": g("TRANS_F32"),
         "F64": g("ADD_F64") + g("MUL_F64") + g("FMA_F64"), "TRANS_F64": g("TRANS_F64"),
         "INT32": g("INT32"), "INT64": g("INT64"), "CVT": g("CVT")}
    n["OTHER"] = max(0.0, c["SQ_INSTS_VALU"] - sum(n.values()))
    need = sum(n[k] * price[k] for k in n)
    return {"counts": n, "price_cycles_4waves": price, "packed_share": PACKED_SHARE,
            "issue_source": "tools/mb/issue_mb.hip at 4 waves/SIMD, ILP 8 (profiles/r05_issue_mb.txt)",
            "simd_cycles_needed": need, "frac_mix": need / (cycles * N_SIMD),
            "formula": "frac_mix = sum_class(count x price) / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)"}


def main():
    out_path, summary, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    per, dur = collect(dirs)
    want = os.environ.get("QKD_PMC_KERNEL")
    names = [k for k in per if (want in k if want else "decode" in k)]
    assert len(names) == 1, names
    with open(summary) as f:
        kernel_ms = [r["warm_avg_ms"] for r in json.load(f)["kernels"] if r["kernel"] == names[0]][0]
    c = {k: sum(v) / len(v) for k, v in per[names[0]].items()}
    n = {k: len(v) for k, v in per[names[0]].items()}
    rec = {"kernel": names[0], "dispatches_per_counter": n, "counters": c,
           "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KB = 1024 B"}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rec["fetch_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        rec["write_bytes"] = c["WRITE_SIZE"] * 1024
        rec["hbm_bytes_per_launch"] = rec["fetch_bytes"] + rec["write_bytes"]
    t = kernel_ms / 1e3
    v = {"kernel_ms": kernel_ms}
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / N_XCD          # summed over the 8 XCDs
        v["gpu_cycles"] = cyc
        # the clock over the counted dispatches' own durations (the PMC pass runs
        # the kernel under other conditions than the trace pass's warm average)
        g = per[names[0]]["GRBM_GUI_ACTIVE"]
        d = dur[names[0]].get("GRBM_GUI_ACTIVE", [])
        if len(d) == len(g) and d and min(d) > 0:
            v["effective_clock_ghz"] = sum(x / N_XCD / y for x, y in zip(g, d)) / len(g)
            v["pmc_pass_kernel_ms"] = sum(d) / len(d) / 1e6
            v["clock_source"] = "GRBM_GUI_ACTIVE / 8 over each counted dispatch's End - Start"
        else:
            v["effective_clock_ghz"] = cyc / t / 1e9
            v["clock_source"] = "GRBM_GUI_ACTIVE / 8 over the trace pass's warm average"
        if "SQ_INSTS_VALU" in c:
            v["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
            v["valu_issue_util_2cyc"] = c["SQ_INSTS_VALU"] * 2 / (cyc * N_SIMD)
        if "SQ_ACTIVE_INST_VALU" in c:
            v["valu_active_util_x4"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * N_SIMD)
    mix = valu_mix(c, v.get("gpu_cycles"))
    if mix:
        v["mix"] = mix
    if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
        v["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
        v["wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_INST_LDS" in c and "SQ_WAVE_CYCLES" in c:
        v["wait_lds_frac"] = c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        v["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    v["formulas"] = ("effective clock: clock_source; valu_issue_util_2cyc = SQ_INSTS_VALU x 2 "
                     "cycles (wave64 over 32 lanes) / (cycles x 1024 SIMDs), binary64 ops take longer; "
                     "valu_active_util_x4 = SQ_ACTIVE_INST_VALU x 4 / (cycles x 1024); lds_conflict_frac = "
                     "SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES")
    rec["valu"] = v
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps({k: rec[k] for k in rec if k != "counters"}))


if __name__ == "__main__":
    main()
