"""Warm per-kernel durations from a rocprofv3 --kernel-trace run:

    python tools/prof_summary.py DIR OUT.json [--skip N]

DIR holds run_kernel_trace.csv. For every kernel name the first N dispatches
(default 3: the bench's warmup and first timed steps pay cold caches and code
loading) are dropped and the rest averaged, so the summary compares with the
bench's warm HIP-event timing."""
import collections
import csv
import json
import os
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 3
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        durs[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for k, v in durs.items():
        v = [x for _, x in sorted(v)]
        warm = v[skip:] if len(v) > skip else v
        rows.append({"kernel": k, "dispatches": len(v), "warm_dispatches": len(warm),
                     "warm_avg_ms": sum(warm) / len(warm) / 1e6, "min_ms": min(v) / 1e6, "max_ms": max(v) / 1e6})
    rows.sort(key=lambda r: -r["warm_avg_ms"] * r["warm_dispatches"])
    with open(out, "w") as f:
        json.dump({"skip_first": skip, "kernels": rows}, f, indent=1)
    for r in rows[:8]:
        print(f"{r['warm_avg_ms']:9.4f} ms x{r['warm_dispatches']:3d}  {r['kernel'][:110]}")


if __name__ == "__main__":
    main()
