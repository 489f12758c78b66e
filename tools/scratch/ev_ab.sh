set -u
cd /root/repo
export TMPDIR=/tmp
for r in 1 2 3; do
for e in on off; do
timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-sweeps --no-e2e --steps 30 --kernel-events $e > gpurun_out/ev_$e.json 2>/dev/null || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/ev_$e.json').read().strip().splitlines()[-1])
print('$e', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['call_ms'],4))"
done; done
