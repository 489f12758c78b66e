set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/syn
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/syn/pytest.log 2>&1; rc=$?
tail -n 3 gpurun_out/syn/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED" gpurun_out/syn/pytest.log | head -60; exit $rc; }
PARITY_K=config2_every_cap REPS=3 bash tools/gpu_ab.sh
