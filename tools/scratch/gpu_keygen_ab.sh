# Key-generation variants (lanes per frame): parity of each build's keygen,
# then the end-to-end line (keygen + decode) of each, alternating.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for l in ${LIBS:-base kg4 kg6}; do
  lib=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; [ $l = base ] || lib=exp_libs/$l/libqkd_ldpc_amd.so
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_large_codes.py tests/test_spec.py -m gpu -q -x \
    --timeout 300 --timeout-method thread -k "keygen or trials" > gpurun_out/kg_parity_$l.log 2>&1; rc=$?
  echo "$l parity rc=$rc $(tail -n 1 gpurun_out/kg_parity_$l.log)"
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for l in ${LIBS:-base kg4 kg6}; do
    lib=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; [ $l = base ] || lib=exp_libs/$l/libqkd_ldpc_amd.so
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --steps 10 > gpurun_out/kg_$l.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/kg_$l.log').read().strip().splitlines()[-1]);print('$l', round(d['ms_per_step'],3), 'e2e', round(d['end_to_end']['ms_per_step'],3), d['end_to_end']['sum_iterations'])"
  done
done
