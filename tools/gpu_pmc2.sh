#!/bin/bash
# Second PMC set: VALU mix, memory pipeline pressure, L2 request latency.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --no-variants"}
k=0
while read -r grp; do
  [ -z "$grp" ] && continue
  k=$((k+1))
  echo "== pmc2 pass $k: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc2_$k" -o run -- python3 bench.py $ARGS > "$OUT/pmc2_$k.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$OUT/pmc2_$k.log"; exit $rc; fi
done <<'PASSES'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU
TA_BUSY_avr TA_ADDR_STALL_CYCLES_sum GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum
SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
PASSES
echo "== done"
