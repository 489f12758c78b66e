#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per run; no
# tracing domains are combined with --pmc). Output: $OUT/pmc_<k>/...
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
  echo "== pmc pass $k: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$k" -o run -- python3 bench.py $ARGS > "$OUT/pmc_$k.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$OUT/pmc_$k.log"; exit $rc; fi
done <<'PASSES'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
PASSES
echo "== done"
