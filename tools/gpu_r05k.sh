# Round-5 call: PMC passes over the long-code bench with the
# frame-interleaved decoder (HBM bytes, waits, VALU).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
k=0
while read -r grp; do
  [ -z "$grp" ] && continue
  k=$((k+1))
  QKD_ILV=1 timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$k -o run -- \
    python3 tools/large_code_bench.py --qber 0.02 > $O/pmc_$k.log 2>&1 || { echo "pass $k failed"; tail $O/pmc_$k.log; exit 1; }
done <<'PASSES'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT
PASSES
echo done
