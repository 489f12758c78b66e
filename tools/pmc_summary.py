"""Average each PMC counter of the decode kernel over its dispatches:
python tools/pmc_summary.py gpurun_out/pmc2_*/run_counter_collection.csv"""
import collections
import csv
import os
import sys

KERNEL = os.environ.get("QKD_PMC_KERNEL", "decode_kernel<1, 0,")   # binary64 keys path
agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:36s} {sum(v) / len(v):18.1f}")
