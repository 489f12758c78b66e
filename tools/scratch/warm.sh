set -u
O=gpurun_out/warm; mkdir -p $O
timeout -k 10 120 python tools/warm_probe.py --blocks 60 --block 5 > $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
cat $O/probe.txt
for w in 5 100 5 100; do
timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-sweeps --no-e2e --steps 20 --warmup $w > $O/b$w.json 2>/dev/null || exit 1
python -c "import json;d=json.loads(open('$O/b$w.json').read().strip().splitlines()[-1]);print('warmup $w step',round(d['ms_per_step'],4),'kernel',round(d['roofline']['kernel_ms'],4),'call',round(d['roofline']['call_ms'],4))"
done
