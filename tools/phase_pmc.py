"""Per-phase PMC table from the phase-stop builds' passes (tools/gpu_phase_pmc.sh).

    python tools/phase_pmc.py OUTDIR [JSON_OUT]

OUTDIR holds <tree>_s<K>_<pass>/run_counter_collection.csv. For each tree the
decode_split_kernel's mean counters per dispatch at every stop K; consecutive
stops are differenced into the phase between them (tools/phase_stop_patch.py
numbers the boundaries). Derived per phase: kernel cycles (GRBM_GUI_ACTIVE / 8),
VALU and SALU instructions, LDS bank-conflict cycles over LDS-active cycles, the
share of wave-cycles spent waiting.
"""
import collections
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import collect  # noqa: E402

FULL = 1000000
PHASES = {0: "frame prologue + epilogue", 3: "iteration 1 (folded: bit phase + syndrome test)",
          4: "iteration 2 check phase (psi)", 5: "iteration 2 bit phase", 6: "iteration 2 syndrome test",
          7: "iteration 3 paired check phase", 8: "iteration 3 bit phase", 9: "iteration 3 syndrome test",
          FULL: "iterations 4+ and exact replays"}


def load(outdir):
    runs = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(glob.glob(os.path.join(outdir, "*_s*_*"))):
        m = re.match(r"(.+)_s(\d+)_(\d+)$", os.path.basename(d))
        if not m or not os.path.isdir(d):
            continue
        runs[(m.group(1), int(m.group(2)))]["dirs"].append(d)
    out = {}
    for (tree, k), v in runs.items():
        per, _ = collect(v["dirs"])
        names = [n for n in per if "decode_split_kernel" in n]
        if len(names) != 1:
            continue
        out.setdefault(tree, {})[k] = {c: sum(x) / len(x) for c, x in per[names[0]].items()}
    return out


def derive(c):
    g = lambda k: c.get(k, 0.0)
    return {"cycles": g("GRBM_GUI_ACTIVE") / 8, "valu": g("SQ_INSTS_VALU"), "salu": g("SQ_INSTS_SALU"),
            "lds_insts": g("SQ_INSTS_LDS"), "lds_conflict_cyc": g("SQ_LDS_BANK_CONFLICT"),
            "lds_active_cyc": g("SQ_LDS_IDX_ACTIVE"), "wait_any": g("SQ_WAIT_ANY"), "wave_cycles": g("SQ_WAVE_CYCLES"),
            "wait_lds": g("SQ_WAIT_INST_LDS"), "lds_atomic": g("SQ_INSTS_LDS_ATOMIC"),
            "lds_load": g("SQ_INSTS_LDS_LOAD"), "lds_store": g("SQ_INSTS_LDS_STORE"),
            "vmem_rd": g("SQ_INSTS_VMEM_RD"), "vmem_wr": g("SQ_INSTS_VMEM_WR"), "branch": g("SQ_INSTS_BRANCH"),
            "salu_cycles": g("SQ_INST_CYCLES_SALU")}


def phases(stops):
    ks = sorted(stops)
    rows, prev = [], None
    for k in ks:
        cur = derive(stops[k])
        d = cur if prev is None else {x: cur[x] - prev[x] for x in cur}
        r = {"stop": k, "phase": PHASES.get(k, f"stop {k}"), **d}
        r["lds_conflict_frac"] = d["lds_conflict_cyc"] / d["lds_active_cyc"] if d["lds_active_cyc"] > 0 else None
        r["wait_frac"] = d["wait_any"] / d["wave_cycles"] if d["wave_cycles"] > 0 else None
        rows.append(r)
        prev = cur
    return rows


def main():
    outdir = sys.argv[1]
    data = load(outdir)
    res = {t: phases(s) for t, s in sorted(data.items())}
    for t, rows in res.items():
        tot = sum(r["cycles"] for r in rows)
        print(f"== {t}: kernel cycles {tot / 1e6:.3f}M (sum over phases)")
        print(f"{'phase':50s} {'cyc%':>6s} {'VALU M':>8s} {'SALU M':>8s} {'LDS M':>7s} {'conf':>6s} {'wait':>6s} "
              f"{'LDSatom M':>9s}")
        for r in rows:
            f = lambda v, p=3: "-" if v is None else f"{v:.{p}f}"
            print(f"{r['phase']:50s} {100 * r['cycles'] / tot:6.1f} {r['valu'] / 1e6:8.2f} {r['salu'] / 1e6:8.2f} "
                  f"{r['lds_insts'] / 1e6:7.2f} {f(r['lds_conflict_frac'])} {f(r['wait_frac'])} "
                  f"{r['lds_atomic'] / 1e6:9.2f}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fo:
            json.dump({"method": "phase-stop builds (tools/phase_stop_patch.py), counters of stop K minus stop K-1 "
                                 "per decode_split_kernel dispatch, config-2 bench batch (4096 frames)",
                       "trees": res, "raw": data}, fo, indent=1)


if __name__ == "__main__":
    main()
