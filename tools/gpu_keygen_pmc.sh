# GPU: PMC record of the key generator (keygen_split_kernel) on the end-to-end path:
# a kernel-trace pass for its warm time, then separate counter passes.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/kgpmc
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-variants --no-sweeps"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 || { tail $O/trace.log; exit 3; }
python3 tools/prof_summary.py $O/trace $O/kernel_summary.json > /dev/null || exit 4
k=0; dirs=""
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  k=$((k+1)); d=$O/pmc_$k
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $d -o run -- $B > $d.log 2>&1 || { tail $d.log; exit 5; }
  dirs="$dirs $d"
done
QKD_PMC_KERNEL=keygen_split python3 tools/pmc_traffic.py $O/pmc_keygen.json $O/kernel_summary.json $dirs
