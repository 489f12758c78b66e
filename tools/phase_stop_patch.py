"""Per-phase PMC attribution (diagnostic builds only, never the product library).

Patches a copy of decode_split.hip so every frame of decode_split_kernel stops
at its K-th phase boundary (-DQKD_PMC_STOP=K): the loop-top test stops before
any iteration at K = 0; then each check phase, bit phase and syndrome test is
one boundary (a folded first iteration's check phase, which does no work, is
one too). For the keys path with the folded first iteration:
    1 (folded check, empty)  2 bit phase 0   3 syndrome test 0
    4 iteration-2 check      5 bit phase 1   6 syndrome test 1
    7 paired check           8 bit phase 2   9 syndrome test 2 ...
A stopped frame leaves through the normal epilogue (its outputs are garbage;
the PMC run checks nothing). The counters of build K minus those of build K-1
are the work of boundary K's phase over the frames that reach it (frames that
finish earlier do identical work in both). tools/gpu_phase_pmc.sh builds and
profiles the stops; tools/phase_pmc.py tabulates them.

    python tools/phase_stop_patch.py <decode_split.hip>     (in place)
"""
import sys

STOP = """
#ifndef QKD_PMC_STOP
#define QKD_PMC_STOP 1000000
#endif
// per-phase PMC stop point (tools/phase_stop_patch.py): the round words and
// checkpoint counts are cleared so the next frame starts clean
#define QKD_STOP_POINT { if (++pmc_ph == (uint32_t)QKD_PMC_STOP) { \\
    if (tid == 0) { ctl[2] = 0; ctl[3] = 0; ctl[4] = 0; ctl[5] = 0; } break; } }
"""


def patch(src: str) -> str:
    reps = [
        ("bool done = false;", "bool done = false; uint32_t pmc_ph = 0;"),
        ("if (it >= a.max_it) break;", "if (it >= a.max_it || QKD_PMC_STOP == 0) break;"),
        ("pc.mark((FOLDS && it < 2 && fold1) ? 5 + (int)it : 1);",
         "pc.mark((FOLDS && it < 2 && fold1) ? 5 + (int)it : 1); QKD_STOP_POINT"),
        ("pc.mark(2);", "pc.mark(2); QKD_STOP_POINT"),
        ("pc.mark(3);", "pc.mark(3); QKD_STOP_POINT"),
    ]
    for old, new in reps:
        n = src.count(old)
        if n != 1:
            raise SystemExit(f"phase_stop_patch: {old!r} found {n} times (want 1)")
        src = src.replace(old, new)
    i = src.index("#include")
    j = src.index("\n", src.rindex("#include", 0, src.index("namespace"))) + 1
    assert i < j
    return src[:j] + STOP + src[j:]


if __name__ == "__main__":
    p = sys.argv[1]
    s = patch(open(p).read())
    open(p, "w").write(s)
    print(f"patched {p}")
