set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for r in 1 2; do
for l in base la23; do
  lib=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; [ $l = base ] || lib=exp_libs/$l/libqkd_ldpc_amd.so
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$lib timeout -k 10 200 python tools/large_code_bench.py --n 40000 --qber 0.02 2>/dev/null | sed "s/^/$l /" || exit 1
done; done
for l in kg5 kg7 kg8; do
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=exp_libs/$l/libqkd_ldpc_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "keygen" > gpurun_out/kg_$l.log 2>&1 || { tail -20 gpurun_out/kg_$l.log; exit 1; }
  echo "$l keygen parity $(tail -n 1 gpurun_out/kg_$l.log)"
done
for r in 1 2; do
for l in base kg5 kg7 kg8; do
  lib=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; [ $l = base ] || lib=exp_libs/$l/libqkd_ldpc_amd.so
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-sweeps --steps 20 > gpurun_out/kgb_$l.json 2>/dev/null || exit 1
  python -c "
import json;d=json.loads(open('gpurun_out/kgb_$l.json').read().strip().splitlines()[-1])
print('$l', 'step', round(d['ms_per_step'],4), 'e2e', round(d['end_to_end']['ms_per_step'],4))"
done; done
