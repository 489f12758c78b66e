# Kernel timeline of the decode-only and end-to-end bench steps.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 tools/e2e_timeline.py \
  > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
python3 tools/e2e_timeline.py --summarise $O/p/run_kernel_trace.csv
