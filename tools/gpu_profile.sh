#!/bin/bash
# Round profile of the shipped decoders (run on the GPU box):
#  1. rocprofv3 --kernel-trace --stats of the bench (every variant), warm per-kernel
#     averages -> $OUT/kernel_summary.json (tools/prof_summary.py)
#  2. per decoder variant, separate --pmc passes (one counter group per run, no trace
#     domains) over a short bench of that variant -> $OUT/pmc_<variant>.json
# Each step has its own time limit; any failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r05prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
VARIANTS=${VARIANTS:-"sp_f64 sp_f32 minsum minsum_sc"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweeps > "$OUT/trace.log" 2>&1 \
  || { tail -n 20 "$OUT/trace.log"; exit 3; }
tail -n 1 "$OUT/trace.log"
python3 tools/prof_summary.py "$OUT/trace" "$OUT/kernel_summary.json" || exit 4
for v in $VARIANTS; do
  dirs=""
  k=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    k=$((k+1))
    d="$OUT/pmc_${v}_$k"
    echo "== $v pass $k: $grp"
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$d" -o run -- \
      python3 bench.py --variant $v --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-e2e --no-sweeps > "$d.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -n 20 "$d.log"; exit $rc; fi
    dirs="$dirs $d"
  done <<'PASSES'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64
SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU
PASSES
  python3 tools/pmc_traffic.py "$OUT/pmc_$v.json" "$OUT/kernel_summary.json" $dirs || exit 5
done
echo "== done"
