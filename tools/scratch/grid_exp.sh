for g in 256 192 128 64; do
  QKD_DECODE_GRID=$g timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --steps 5 > gpurun_out/grid_$g.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/grid_$g.json').read().strip().splitlines()[-1]); print($g, round(d['roofline']['kernel_ms'],3), round(d['roofline']['kernel_ms']*$g/256,3))"
done
