set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/kgpmc; mkdir -p $O
i=0
while read -r grp; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 tools/kg_probe.py 20 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 3; }
done <<'P'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT
P
python3 - <<'PY'
import csv, glob, collections
acc=collections.defaultdict(list)
for f in glob.glob("gpurun_out/kgpmc/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "keygen_split" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in sorted(acc.items()):
    # per-dispatch values may be split per XCD/SE rows: sum by dispatch is approximate; print mean of rows x rows/dispatch
    print(k, len(v), sum(v)/20)
PY
