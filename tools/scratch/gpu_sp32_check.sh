set -u
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_variants.py tests/test_spec.py -m gpu -q -x --timeout 300 --timeout-method thread -k "variant or sp32 or f32 or phi_pair" > gpurun_out/pytest_sp32.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_sp32.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 120 python bench.py --variant sp_f32 --no-cpu-baseline --no-variants --no-e2e --steps 20 > gpurun_out/b32.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/b32.log').read().strip().splitlines()[-1]);print('sp_f32', d['ms_per_step'], d['roofline']['kernel_ms'], d['fer'], d['mean_iterations'])"
done
timeout -k 10 600 python tools/minsum_sweep.py --trials 100000 --qbers 0.07,0.08 > gpurun_out/minsum_sweep.jsonl 2> gpurun_out/minsum_sweep.err || exit $?
