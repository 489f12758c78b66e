set -u
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -n 15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_split.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_split.log
QKD_DECODE_KERNEL=classic timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_classic.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_classic.log
QKD_PHASE_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants > gpurun_out/phase.log 2>&1; tail -c 400 gpurun_out/phase.log
exit $rc
