"""Time the oracle (oracle/oracle.c, the CPU restatement used as bench.py's
cpu_baseline) on config 2 with 8 threads, in the build container whose 8-core Xeon
the survey timed the reference on (2.66-2.76 s), and record it in
profiles/cpu_calibration.json for bench.py's calibration ratio.

    python tools/cpu_calibrate.py [--repeat 3]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    O.build()
    code = O.Code.from_lists(dict(np.load(os.path.join(ROOT, "tests", "golden", "code_n10240.npz"))))
    seeds = O.seeds(777, 4096)
    times = []
    for _ in range(args.repeat):
        t0 = time.perf_counter()
        r = code.trials(0.02, seeds, 0, 50, 100.0, True, threads=args.threads)
        times.append(time.perf_counter() - t0)
    assert int(r["iters"].sum()) == 12905
    cpu = ""
    try:
        cpu = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:
        pass
    rec = {"oracle_c2_seconds": min(times), "all_runs_s": times, "threads": args.threads,
           "host": f"{cpu} ({os.cpu_count()} CPUs), {platform.platform()}",
           "reference_c2_seconds": [2.66, 2.76],
           "reference_source": "SURVEY.md §6: reference batch mode, g++ -O3, 8 threads, same container type",
           "ratio_oracle_over_reference": min(times) / 2.71}
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
