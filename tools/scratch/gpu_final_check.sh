# Round-end check on one GPU: the whole -m gpu suite, smoke, the headline bench
# (with the CPU baseline), the config-4 per-rank share (125,000 frames).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print('headline', round(d['value']/1e9,2), 'Gbit/s', round(d['ms_per_step'],3), 'ms; e2e', round(d['end_to_end']['ms_per_step'],3), {k: round(v['kernel_ms'],3) for k,v in d['variants'].items()})"
timeout -k 10 300 python bench.py --frames 125000 --steps 5 --warmup 1 --no-cpu-baseline --no-variants --no-e2e > gpurun_out/bench_c4share.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_c4share.log').read().strip().splitlines()[-1]);print('c4 share', round(d['value']/1e9,2), 'Gbit/s', round(d['ms_per_step'],2), 'ms', d['fer'], d['mean_iterations'])"
