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
# profiles/r06_issue_mb.txt (one row per opcode the decoder issues). Each PMC
# class (SQ_INSTS_VALU_<class>; OTHER = the rest of SQ_INSTS_VALU) is priced at
# the mean cost of ITS opcodes weighted by the decoder's dynamic opcode census
# (tools/valu_census.py: the kernel's ISA split into phases, each phase's
# innermost-loop mix scaled to the per-phase PMC VALU count; committed as
# profiles/r*_valu_census.json). So packed and scalar binary32 FMAs, and the
# selects, moves, shifts, compares and lane reads of OTHER, each count at their
# own measured cost in the proportion the kernel executes them.
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import valu_census  # noqa: E402

PROFILES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
PMC_CLASSES = ("FMA_F32", "MUL_F32", "ADD_F32", "TRANS_F32", "F64", "TRANS_F64", "INT32", "INT64", "CVT")


def newest(pattern):
    import glob
    fs = sorted(glob.glob(os.path.join(PROFILES, pattern)))
    return fs[-1] if fs else None


def pmc_class_counts(c):
    """The PMC record's VALU instructions per class; OTHER = the unclassified rest."""
    g = lambda k: c.get("SQ_INSTS_VALU_" + k, 0.0)
    n = {"FMA_F32": g("FMA_F32"), "MUL_F32": g("MUL_F32"), "ADD_F32": g("ADD_F32"), "TRANS_F32": g("TRANS_F32"),
         "F64": g("ADD_F64") + g("MUL_F64") + g("FMA_F64"), "TRANS_F64": g("TRANS_F64"),
         "INT32": g("INT32"), "INT64": g("INT64"), "CVT": g("CVT")}
    n["OTHER"] = max(0.0, c["SQ_INSTS_VALU"] - sum(n.values()))
    return n


def census_prices(census_path=None, issue_path=None):
    """{class: cycles} from the committed census and issue table; a class the
    census does not see (or with no measured opcode) takes the FMA_F32 price
    for F64 work's 2x and the census-wide mean otherwise."""
    census_path = census_path or newest("r*_valu_census.json")
    issue_path = issue_path or newest("r*_issue_mb.txt")
    rec = json.load(open(census_path))
    costs = valu_census.load_costs(issue_path)
    cp = valu_census.class_prices(rec["dynamic_per_launch"], costs)
    tot = sum(v["count"] for v in cp.values() if v["cycles"])
    mean = sum(v["count"] * v["cycles"] for v in cp.values() if v["cycles"]) / tot
    price = {k: (cp[k]["cycles"] if k in cp and cp[k]["cycles"] else mean) for k in PMC_CLASSES + ("OTHER",)}
    if not (cp.get("TRANS_F64") or {}).get("cycles"):
        price["TRANS_F64"] = 2 * costs.get("v_fma_f64", mean)
    return price, cp, os.path.basename(census_path), os.path.basename(issue_path)


def valu_mix(c, cycles, census_path=None, issue_path=None):
    """The PMC record's VALU classes priced at their census-weighted 4-wave issue
    costs: the SIMD-cycles the kernel's VALU stream needs, and the share of the
    kernel's SIMD-cycles that is (frac_mix, the issue-bound fraction at the
    kernel's own instruction mix)."""
    if "SQ_INSTS_VALU" not in c or not cycles:
        return None
    price, cp, csrc, isrc = census_prices(census_path, issue_path)
    n = pmc_class_counts(c)
    need = sum(n[k] * price[k] for k in n)
    return {"counts": n, "price_cycles_4waves": price,
            "census": {k: {"count": v["count"], "measured_share": v["measured_share"]} for k, v in cp.items()},
            "census_source": "profiles/" + csrc, "issue_source": "profiles/" + isrc,
            "simd_cycles_needed": need, "frac_mix": need / (cycles * N_SIMD),
            "formula": "frac_mix = sum_class(PMC count x census-weighted 4-wave cost of the class's opcodes) / "
                       "(GRBM_GUI_ACTIVE/8 x 1024 SIMDs)"}


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
