set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED" $O/pytest_gpu.log | head -80; exit $rc; }
bash tools/gpu_ab.sh
