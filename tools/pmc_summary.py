"""Average each PMC counter of the decode kernel over its dispatches:
python tools/pmc_summary.py gpurun_out/pmc2_*/run_counter_collection.csv"""
import collections
import csv
import sys

agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        if "decode_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:36s} {sum(v) / len(v):18.1f}")
