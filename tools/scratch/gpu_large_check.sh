# GPU check of long codes: parity of both kernels, then the throughput of the
# split-store and classic kernels on a random (3,6)-regular N = 40000 code, and
# the headline A/B against a given build ($AB_LIB).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_large_codes.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_large.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_large.log
[ $rc -eq 0 ] || exit $rc
for q in 0.02 0.03 0.05; do
  timeout -k 10 300 python tools/large_code_bench.py --n 40000 --qber $q > gpurun_out/large_split_$q.json || exit $?
  cat gpurun_out/large_split_$q.json
done
QKD_DECODE_KERNEL=classic timeout -k 10 300 python tools/large_code_bench.py --n 40000 --qber 0.03 > gpurun_out/large_classic.json || exit $?
cat gpurun_out/large_classic.json
if [ -n "${AB_LIB:-}" ]; then
  REPS=3 SWEEP="old QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$AB_LIB
new" bash tools/gpu_env_sweep.sh || exit $?
fi
