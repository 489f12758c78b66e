#!/bin/bash
# GPU quick check: parity tests, then the bench with phase timing.
set -u
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -n 15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
QKD_PHASE_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench.log
