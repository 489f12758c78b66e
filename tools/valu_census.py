"""Dynamic VALU opcode census of the headline decoder, for pricing its VALU issue.

The static ISA (hipcc --save-temps of decode_split.hip, tools/isa_census.py's
input) is split into the decoder's phases by source line: every instruction
belongs to the phase of the last decode_split.hip line the .loc directives named
before it (helpers inlined from other files, and decode_split.hip's own small
helpers above the phase functions, inherit that context). Inside each phase the
instructions of its innermost hot loops (at least MIN_LOOP_VALU VALU
instructions: a task or a bit round) stand for its dynamic mix (the loop
bodies execute once per task / bit batch; the straight-line code around them
once per phase). Each phase's mix is then scaled to the VALU count the per-phase PMC
record measured for it (tools/phase_pmc.py: phase-stop builds, counters of stop
K minus stop K - 1), which gives dynamic counts per opcode.

The per-opcode counts are checked against the whole-kernel PMC classes
(SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F32, INT32, ...), and priced at the 4-wave
issue costs tools/mb/issue_mb.hip measures per opcode (profiles/r06_issue_mb.txt).

    python tools/valu_census.py census KERNEL.s PHASE_PMC.json OUT.json
    (tools/census_isa.sh OUT.s PHASE_PMC.json OUT.json builds KERNEL.s first)
    python tools/valu_census.py variant KERNEL.s VARIANT W_CHECK W_BIT OUT.json

Round 6 (profiles/r06_valu_census.json, from profiles/r06_phase_pmc.json): of
592M VALU per config-2 launch 306M are OTHER, led by v_cndmask_b32 (82M: the
interval selects -- neg_iv_if's swapped negation, the x < 1 branch selects of
phi_core, the certified / uncertified masks), v_lshrrev_b32 (21M), v_mov_b32
(19M), v_and_b32 (16M), v_bfe_u32 (16M: plan-word fields), v_med3_f32 /
v_cmp_gt_f32 (15M each: clamps and the interval tests), v_max_f32 (13M),
v_readfirstlane / v_readlane (10M each: uniform task indices and SGPR spills).
"""
from __future__ import annotations

import collections
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "decode_split_kernelILi1ELi0ELi6ELb1ELi1ELb0E"   # keys path, binary64, DC 6, clamp, speculative
SRC = "decode_split.hip"

# (first, last) decode_split.hip lines of each phase function / kernel part;
# lines below HELPERS_END are small helpers inlined everywhere (they inherit)
HELPERS_END = 283


def regions(src_path):
    """Line ranges of the phase functions, found by their signatures in the source
    (so the table follows the file as it changes)."""
    lines = open(src_path).read().splitlines()
    starts = {}
    pats = {
        "exact_check": r"__device__ __forceinline__ void split_check_phase\(",
        "sp32_check": r"__device__ __forceinline__ void sp32_check_phase\(",
        "ms_check": r"__device__ __forceinline__ void ms_split_check_phase\(",
        "sp32_bit": r"__device__ __forceinline__ void sp32_bit_phase\(",
        "check_psi": r"__device__ __forceinline__ void spec_check_phase_psi\(",
        "check_paired": r"__device__ __forceinline__ void spec_check_phase_paired\(",
        "fold_fill": r"__device__ void fold_table_fill\(",
        "bit": r"__device__ __forceinline__ void spec_bit_phase\(",
        "kernel_setup": r"void decode_split_kernel\(DecodeArgs a\)",
        "prologue": r"// ---- prologue\. Keys path",
        "iteration": r"// ---- iterations \(",
        "epilogue": r"// ---- outputs: SP_result",
        "host": r"__global__ __launch_bounds__\(kSynBlock\) void frame_syn_kernel",
    }
    for name, p in pats.items():
        for i, l in enumerate(lines, 1):
            if re.search(p, l):
                starts[name] = i
                break
    order = sorted(starts.items(), key=lambda kv: kv[1])
    out = []
    for k, (name, s) in enumerate(order):
        e = order[k + 1][1] - 1 if k + 1 < len(order) else len(lines)
        out.append((name, s, e))
    return out


def region_of(line, table):
    for name, s, e in table:
        if s <= line <= e:
            return name
    return None


def kernel_body(path, pat):
    files, out, on = {}, [], False
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
        if not on and line.startswith("_Z") and pat in line.split(":")[0]:
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return files, out


def opcode(line):
    return re.sub(r"_e(32|64|64_dpp|32_dpp|_sdwa)$", "", line.split()[0])


def parse(path, pat, table):
    """[(opcode, region, index)] of the kernel's instructions, and the loops as
    (header index, back-edge index) over that list."""
    files, body = kernel_body(path, pat)
    ins, labels, ctx = [], {}, None
    branches = []
    for l in body:
        m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            f, ln = files.get(m.group(1), m.group(1)), int(m.group(2))
            if f == SRC and ln >= HELPERS_END:
                r = region_of(ln, table)
                if r:
                    ctx = r
            continue
        if l.startswith(".LBB"):
            labels[l.split(":")[0]] = len(ins)
            continue
        if not l.startswith("\t") or l.strip().startswith((";", ".")) or not l.strip():
            continue
        o = opcode(l.strip())
        if o.startswith(("s_cbranch", "s_branch")):
            branches.append((len(ins), l.split()[-1]))
        ins.append((o, ctx))
    loops = [(labels[t], i) for i, t in branches if t in labels and labels[t] <= i]
    return ins, loops


def innermost(loops, ins=None, min_valu=0):
    """Loops that contain no other loop. With ins and min_valu: among the loops
    of at least min_valu VALU instructions only (a phase's batch loop counts as
    innermost around the few-instruction loops the compiler leaves inside it --
    exec-mask waterfalls, zero fills -- which themselves are dropped)."""
    if ins is not None and min_valu:
        loops = [(a, b) for a, b in loops if sum(1 for o, _ in ins[a:b + 1] if o.startswith("v_")) >= min_valu]
    out = []
    for a, b in loops:
        if not any((c, d) != (a, b) and a <= c and d <= b for c, d in loops):
            out.append((a, b))
    return out


# a hot loop has at least this many VALU instructions (one task or bit round)
MIN_LOOP_VALU = 40


# SQ_INSTS_VALU_* class of an opcode: the PMC's own classes (packed binary32
# FMA / MUL / ADD count once, as their scalar forms), INT32 = integer
# arithmetic, INT64 = 64-bit integer shifts and adds, CVT = conversions; the
# rest (selects, compares, moves, logic, 32-bit shifts, bit fields, min / max /
# med3, lane reads) is what tools/pmc_traffic.py calls OTHER
def pmc_class(o):
    if re.match(r"v_(pk_)?(fma|fmac|mad|mac|fmamk|fmaak)_f32", o):
        return "FMA_F32"
    if re.match(r"v_(pk_)?mul_f32", o):
        return "MUL_F32"
    if re.match(r"v_(pk_)?(add|sub|subrev)_f32", o):
        return "ADD_F32"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", o):
        return "TRANS_F32"
    if re.match(r"v_(rcp|rsq|sqrt)_f64", o):
        return "TRANS_F64"
    if re.match(r"v_(fma|add|mul)_f64", o):
        return "F64"
    if re.match(r"v_cvt_", o):
        return "CVT"
    if re.match(r"v_(lshrrev|lshlrev|ashrrev)_[bi]64|v_lshl_add_u64|v_mad_[ui]64", o):
        return "INT64"
    if re.match(r"v_(add|sub|subrev|add3|mul_lo|mul_hi|mad|lshl_add|add_lshl|add_co|sub_co|addc_co|subb_co)_"
                r"(u32|i32|u16|i16|u32_u24|i32_i24|co_u32)", o):
        return "INT32"
    return "OTHER"


def load_costs(path=os.path.join(ROOT, "profiles", "r06_issue_mb.txt"), waves=4.0, ilp=8):
    """{measured name: shader cycles per wave-instruction per SIMD} at the
    decoder's occupancy (tools/mb/issue_mb.hip)."""
    out = {}
    for line in open(path):
        f = line.split()
        if len(f) == 7 and float(f[2]) == waves and int(f[4]) == ilp:
            out[f[0]] = float(f[6])
    return out


# opcodes priced by a measured one of the same encoding and operand shape
ALIAS = [
    (r"v_cndmask_b32", "v_cndmask_b32_sgpr"),     # see opcode_cost
    (r"v_fmaak_f32|v_fmamk_f32", "v_fmamk_f32"),
    (r"v_fmac_f32|v_mac_f32|v_fma_f32|v_mad_f32", "v_fma_f32"),
    (r"v_cmp\w*_f32", "v_cmp_gt_f32"),
    (r"v_cmp\w*_f64", "v_cmp_lt_f64"),
    (r"v_cmp\w*_[ui](16|32|64)", "v_cmp_ne_u32"),
    (r"v_(lshrrev|lshlrev|ashrrev)_[bi](16|32)", "v_lshrrev_b32"),
    (r"v_(lshrrev|lshlrev|ashrrev)_[bi]64|v_lshl_add_u64", "v_lshrrev_b64"),
    (r"v_(sub|subrev|add_co|sub_co|addc_co|subb_co)_u32|v_add_u32|v_add_i32", "v_add_u32"),
    (r"v_(add|sub)_[ui]16", "v_add_u16"),
    (r"v_mul_lo_u16", "v_mul_lo_u16"),
    (r"v_(mad|mul)_u32_u24|v_mad_i32_i24|v_mul_u32_u24|v_mul_lo_u32", "v_mad_u32_u24"),
    (r"v_lshl_add_u32|v_add_lshl_u32|v_add3_u32|v_lshl_or_b32|v_and_or_b32|v_or3_b32", "v_lshl_add_u32"),
    (r"v_bfe_[ui]32", "v_bfe_u32"),
    (r"v_bfi_b32|v_perm_b32|v_alignbit_b32|v_alignbyte_b32", "v_bfi_b32"),
    (r"v_(max|min)\w*_(f32|u32|i32)", "v_max_f32"),
    (r"v_med3_\w+", "v_med3_f32"),
    (r"v_not_b32|v_xor_b32", "v_xor_b32"),
    (r"v_bcnt_u32_b32|v_mbcnt_\w+", "v_bcnt_u32_b32"),
    (r"v_mov_b64|v_pk_mov_b32", "v_pk_mov_b32"),
    (r"v_writelane_b32|v_readlane_b32", "v_readlane_b32"),
    (r"v_cvt_\w+", "v_cvt_f32_f64"),
    (r"v_(rsq|sqrt)_f32", "v_rcp_f32"),
    (r"v_(fma|mul|fmac)_f64|v_div_\w+_f64|v_(min|max)_f64", "v_fma_f64"),
    (r"v_(sub|subrev)_f32", "v_add_f32"),
    (r"v_bitop3_b(16|32)", "v_bfi_b32"),        # gfx950's three-input bit operation (VOP3, 3 sources)
]


def opcode_cost(o, costs):
    """(cycles, the measured entry used). Selects: the VOP3 and VOP2 forms cost
    the same among other VALU work (issue_mb's 3fma+cndmask_e32 / _e64 rows); the
    VOP2 form's 19 cycles is back-to-back VCC selects only, which the decoder's
    schedule never issues, so every select is priced as the measured SGPR-mask
    form."""
    base = re.sub(r"_sdwa$", "", o)
    if o.endswith("_sdwa") and "v_lshrrev_b32_sdwa" in costs:
        return costs["v_lshrrev_b32_sdwa"], "v_lshrrev_b32_sdwa"
    for pat, name in ALIAS:
        if re.fullmatch(pat, base) and name in costs:
            return costs[name], name
    if base in costs:
        return costs[base], base
    return None, None


def class_prices(dyn, costs):
    """Per PMC class: the census-weighted mean of its opcodes' measured costs,
    the class's dynamic count, and the share of it priced by a measured
    opcode (an unmeasured opcode takes its class's mean)."""
    acc = collections.defaultdict(lambda: [0.0, 0.0, 0.0])   # count, priced count, priced cycles
    for o, n in dyn.items():
        if not o.startswith("v_"):
            continue
        c, _ = opcode_cost(o, costs)
        a = acc[pmc_class(o)]
        a[0] += n
        if c is not None:
            a[1] += n
            a[2] += n * c
    return {k: {"count": v[0], "measured_share": v[1] / v[0] if v[0] else 0.0,
                "cycles": v[2] / v[1] if v[1] else None} for k, v in acc.items()}


def load_phases(path, tree=None):
    """(tree, [{"phase", "valu"}]) from tools/phase_pmc.py's JSON or its text table
    (the last tree, or the named one)."""
    if path.endswith(".json"):
        ph = json.load(open(path))
        t = tree or sorted(ph["trees"])[-1]
        return t, ph["trees"][t]
    trees, cur = {}, None
    for l in open(path):
        m = re.match(r"== (\S+):", l)
        if m:
            cur = m.group(1)
            trees[cur] = []
            continue
        f = l.rstrip("\n")
        if cur and len(f) > 50 and not f.startswith(("phase", "#")):
            cols = f[50:].split()
            trees[cur].append({"phase": f[:50].strip(), "valu": float(cols[1]) * 1e6})
    t = tree or list(trees)[-1]
    return t, trees[t]


def census(s_path, phase_json, out_path, src_path=None):
    src_path = src_path or os.path.join(ROOT, "qkd_ldpc_amd", "csrc", SRC)
    table = regions(src_path)
    ins, loops = parse(s_path, KERNEL, table)
    inner = innermost(loops, ins, MIN_LOOP_VALU)
    # per region: static counts of the innermost-loop instructions (hot) and of all
    hot = collections.defaultdict(collections.Counter)
    allc = collections.defaultdict(collections.Counter)
    in_loop = [False] * len(ins)
    for a, b in inner:
        for i in range(a, b + 1):
            in_loop[i] = True
    for i, (o, r) in enumerate(ins):
        if not o.startswith("v_"):
            continue
        allc[r][o] += 1
        if in_loop[i]:
            hot[r][o] += 1
    tree, rows = load_phases(phase_json)
    # phase-stop rows -> census regions (tools/phase_pmc.py PHASES)
    valu = {r["phase"]: r["valu"] for r in rows}
    get = lambda key: sum(v for k, v in valu.items() if k.startswith(key))
    weights = {
        "prologue+epilogue": (get("frame prologue"), {"prologue": 1.0, "epilogue": 1.0}),
        "iteration 1 (folded bit phase)": (get("iteration 1"), {"bit": 1.0}),
        "check psi": (get("iteration 2 check"), {"check_psi": 1.0}),
        "bit phases 2-3": (get("iteration 2 bit") + get("iteration 3 bit"), {"bit": 1.0}),
        "syndrome tests": (get("iteration 2 syndrome") + get("iteration 3 syndrome"), {"iteration": 1.0}),
        "check paired": (get("iteration 3 paired"), {"check_paired": 1.0}),
        # iterations 4+ and exact replays: paired check + bit phase in the
        # proportion of iterations 3's, plus the exact rule's check phase
        "iterations 4+ / replays": (get("iterations 4+"), {"check_paired": 0.6, "bit": 0.25, "exact_check": 0.15}),
    }
    dyn = collections.Counter()
    parts = {}
    for name, (count, mix) in weights.items():
        if count <= 0:
            continue
        vec = collections.Counter()
        for reg, w in mix.items():
            src = hot[reg] if sum(hot[reg].values()) else allc[reg]
            tot = sum(src.values())
            if not tot:
                continue
            for o, n in src.items():
                vec[o] += w * n / tot
        s = sum(vec.values())
        for o in vec:
            vec[o] *= count / s
        dyn.update(vec)
        parts[name] = {"valu": count, "top": dict(vec.most_common(8))}
    rec = {"kernel": KERNEL, "s_file": os.path.basename(s_path), "phase_pmc": os.path.basename(phase_json),
           "tree": tree, "regions": table, "innermost_loops": len(inner),
           "static_hot": {r: dict(c) for r, c in hot.items()},
           "phases": parts, "dynamic_per_launch": dict(dyn.most_common())}
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=1)
    return rec


# The binary32 variants (no per-phase PMC record): their kernels' check- and
# bit-phase innermost-loop mixes weighted by the phases' shader-clock shares
# (bench.py --phase-timing, profiles/r06_variants.txt) -- a coarser census
VARIANTS = {
    "sp_f32": ("decode_split_kernelILi1ELi1ELi6ELb1ELi0ELb0E", ("sp32_check",), ("sp32_bit",)),
    "minsum": ("decode_split_kernelILi1ELi5ELi6ELb1ELi0ELb0E", ("ms_check",), ("sp32_bit",)),
    "minsum_sc": ("decode_split_kernelILi1ELi6ELi6ELb1ELi0ELb0E", ("ms_check",), ("sp32_bit",)),
}


def census_variant(s_path, variant, w_check, w_bit, out_path, src_path=None):
    src_path = src_path or os.path.join(ROOT, "qkd_ldpc_amd", "csrc", SRC)
    sym, creg, breg = VARIANTS[variant]
    table = regions(src_path)
    ins, loops = parse(s_path, sym, table)
    in_loop = [False] * len(ins)
    for a, b in innermost(loops, ins, MIN_LOOP_VALU):
        for i in range(a, b + 1):
            in_loop[i] = True
    mix = {}
    for regs, w in ((creg, w_check), (breg, w_bit)):
        c = collections.Counter(o for i, (o, r) in enumerate(ins) if in_loop[i] and r in regs and o.startswith("v_"))
        tot = sum(c.values())
        for o, n in c.items():
            mix[o] = mix.get(o, 0.0) + w * n / tot
    rec = {"kernel": sym, "variant": variant, "s_file": os.path.basename(s_path),
           "weights": {"check": w_check, "bit": w_bit, "source": "phase shader-clock shares, profiles/r06_variants.txt"},
           "dynamic_per_launch": dict(sorted(mix.items(), key=lambda kv: -kv[1])),
           "note": "relative mix only (sums to the weights' total): pricing takes composition, not counts"}
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=1)
    return rec


def main(argv):
    if argv[1] == "variant":
        rec = census_variant(argv[2], argv[3], float(argv[4]), float(argv[5]), argv[6])
        costs = load_costs()
        for k, v in sorted(class_prices(rec["dynamic_per_launch"], costs).items(), key=lambda kv: -kv[1]["count"]):
            print(f"  {k:10s} {v['count']:8.3f}  {v['cycles'] or 0:5.2f} cyc  measured {v['measured_share']:.3f}")
        return
    if argv[1] == "census":
        rec = census(argv[2], argv[3], argv[4])
        tot = sum(rec["dynamic_per_launch"].values())
        print(f"{rec['kernel']}: {rec['innermost_loops']} innermost loops, {tot / 1e6:.1f}M VALU per launch")
        costs = load_costs()
        for k, v in sorted(class_prices(rec["dynamic_per_launch"], costs).items(), key=lambda kv: -kv[1]["count"]):
            print(f"  {k:10s} {v['count'] / 1e6:8.1f}M  {v['cycles'] or 0:5.2f} cyc  measured {v['measured_share']:.3f}")
        for o, n in list(rec["dynamic_per_launch"].items())[:40]:
            c, name = opcode_cost(o, costs)
            print(f"  {o:28s} {n / 1e6:8.2f}M  {pmc_class(o):9s} {c if c else '-':>5} {name or ''}")


if __name__ == "__main__":
    main(sys.argv)
