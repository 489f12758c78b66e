set -u
cd /root/repo
mkdir -p gpurun_out/pmcab
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/pmcab/avail.txt 2>&1 || true
for l in head pair; do
  if [ $l = head ]; then export QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=exp_libs/head/libqkd_ldpc_amd.so; else unset QKD_AMD_LIB; fi
  k=0
  while read -r grp; do
    k=$((k+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcab/${l}_$k -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-e2e > gpurun_out/pmcab/${l}_$k.log 2>&1 || exit $?
  done <<'PASSES'
SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU
SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
PASSES
done
python3 - <<'PY'
import csv,glob,collections,os
for l in ("head","pair"):
    c=collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmcab/{l}_*/**/*counter_collection.csv",recursive=True):
        for r in csv.DictReader(open(f)):
            if "decode_split" in r["Kernel_Name"]: c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(l, {k: "%.4g" % (sum(v)/len(v)) for k,v in sorted(c.items())})
PY
