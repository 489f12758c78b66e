# Per-phase PMC (run on the GPU box): for every phase-stop build in exp_libs/*_s<K>/
# (tools/phase_stop_build.sh), two rocprofv3 --pmc passes (no trace domains) over a
# short config-2 bench; tools/phase_pmc.py differences consecutive stops.
# Every step has its own time limit; a failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/phase_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
for d in exp_libs/*_s*; do
  b=$(basename $d)
  k=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    k=$((k+1))
    o="$OUT/${b}_$k"
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$d/libqkd_ldpc_amd.so timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv \
      -d "$o" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-e2e --no-sweeps \
      > "$o.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$b pass $k rc=$rc"; tail -n 20 "$o.log"; exit $rc; fi
  done <<'PASSES'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE
SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE
PASSES
  echo "$b done"
done
python3 tools/phase_pmc.py "$OUT" > "$OUT/phase_pmc.txt" && cat "$OUT/phase_pmc.txt"
