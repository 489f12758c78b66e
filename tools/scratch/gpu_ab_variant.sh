# A/B of the in-tree build against $AB_LIB: parity subset, then the headline and
# the sp_f32 variant, alternating builds, REPS rounds.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_spec.py tests/test_gpu_parity.py tests/test_variants.py -m gpu -q -x --timeout 300 \
  --timeout-method thread -k "${PARITY_K:-config2 or fresh or bits_match or qkd_ldpc_tables or phi_pair or sp_f32}" > gpurun_out/ab_parity.log 2>&1; rc=$?
echo "parity rc=$rc $(tail -n 1 gpurun_out/ab_parity.log)"
[ $rc -eq 0 ] || exit $rc
for v in sp_f64 sp_f32; do
  REPS=${REPS:-3} BENCH_EXTRA="--variant $v" SWEEP="old_$v QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$AB_LIB
new_$v" bash tools/gpu_env_sweep.sh || exit $?
done
