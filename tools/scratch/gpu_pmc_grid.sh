# PMC of the headline decoder at full occupancy and with QKD_DECODE_GRID capped
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/pmcgrid
export TMPDIR=/tmp
for g in ${GRIDS:-256 128}; do
  k=0
  while read -r grp; do
    k=$((k+1))
    QKD_DECODE_GRID=$g timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcgrid/g${g}_$k -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-e2e > gpurun_out/pmcgrid/g${g}_$k.log 2>&1 || exit $?
  done <<'PASSES'
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum
PASSES
done
python3 - <<'PY'
import csv,glob,collections,os
for g in os.environ.get("GRIDS","256 128").split():
    c=collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmcgrid/g{g}_*/**/*counter_collection.csv",recursive=True):
        for r in csv.DictReader(open(f)):
            if "decode_split" in r["Kernel_Name"]: c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(g, {k: "%.4g" % (sum(v)/len(v)) for k,v in sorted(c.items())})
PY
