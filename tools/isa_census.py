"""ISA census of one kernel's loops in a hipcc --save-temps .s file.

For every backward branch (a loop back edge) prints the loop's span, its
instruction count by class and the opcodes that matter for the decoder's
pricing (readlane / writelane from SGPR spills, transcendentals, packed FMAs,
LDS and buffer accesses). Used to attribute the headline decoder's VALU
(DESIGN.md §4.3):

  python tools/isa_census.py file.s [kernel-symbol-substring] [--min N]
"""
from __future__ import annotations

import collections
import re
import sys

KEYS = ["v_readlane_b32", "v_writelane_b32", "v_readfirstlane_b32", "v_cndmask_b32", "v_mov_b32",
        "v_exp_f32", "v_log_f32", "v_pk_fma_f32", "v_fma_f32", "v_fma_f64", "ds_read", "ds_write",
        "ds_xor", "ds_or", "buffer_load", "buffer_store", "s_waitcnt", "s_cbranch_execz"]


FILES: dict[str, str] = {}


def kernel_lines(path: str, pat: str) -> tuple[str, list[str]]:
    out, name, on = [], "", False
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            FILES[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
        if not on and line.startswith("_Z") and pat in line.split(":")[0]:
            on, name = True, line.split(":")[0]
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return name, out


def op(line: str) -> str:
    o = line.split()[0]
    return re.sub(r"_e(32|64)$", "", o)


def census(lines: list[str]):
    pos = {l.split(":")[0]: i for i, l in enumerate(lines) if l.startswith(".LBB")}
    loops = []
    for i, l in enumerate(lines):
        t = l.split()
        if t and (t[0].startswith("s_cbranch") or t[0] == "s_branch") and t[-1] in pos and pos[t[-1]] < i:
            body = [op(x) for x in lines[pos[t[-1]]:i + 1]
                    if x.startswith("\t") and not x.strip().startswith((";", "."))]
            c = collections.Counter(body)
            locs = collections.Counter()
            for x in lines[pos[t[-1]]:i + 1]:
                m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", x)
                if m:
                    locs[(FILES.get(m.group(1), m.group(1)), int(m.group(2)))] += 1
            row = {"from": pos[t[-1]], "to": i, "n": len(body),
                   "src": " ".join(f"{f}:{l}" for (f, l), _ in sorted(locs.items(), key=lambda kv: -kv[1])[:3]),
                   "v": sum(n for k, n in c.items() if k.startswith("v_")),
                   "s": sum(n for k, n in c.items() if k.startswith("s_"))}
            for k in KEYS:
                row[k] = sum(n for kk, n in c.items() if kk.startswith(k))
            loops.append(row)
    return loops


def main(argv):
    path = argv[1]
    pat = argv[2] if len(argv) > 2 and not argv[2].startswith("--") else "decode_split_kernelILi1ELi0ELi6ELb1ELi1E"
    mn = int(argv[argv.index("--min") + 1]) if "--min" in argv else 60
    name, lines = kernel_lines(path, pat)
    print(name)
    ins = [op(x) for x in lines if x.startswith("\t") and not x.strip().startswith((";", "."))]
    c = collections.Counter(ins)
    print("total", len(ins), {k: sum(n for kk, n in c.items() if kk.startswith(k)) for k in KEYS[:5]})
    hdr = ["from", "to", "n", "v", "s"] + KEYS
    print(" ".join(h.replace("v_", "").replace("_b32", "")[:9] for h in hdr))
    for r in census(lines):
        if r["n"] >= mn:
            print(" ".join(str(r[h]) for h in hdr), "|", r["src"])


if __name__ == "__main__":
    main(sys.argv)
