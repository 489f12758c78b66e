# Long-code frames-in-flight sweep (profiles/r04_large_code_grid.jsonl):
# tools/large_code_bench.py (random (3,6) N = 40000, 4096 frames, QBER 0.02) at
# several QKD_DECODE_GRID caps on the GPU box; each run has its own time limit.
set -u
mkdir -p gpurun_out/lc
for g in 256 192 128 96 64; do
  timeout -k 10 120 python tools/large_code_bench.py --qber 0.02 --debug-opt QKD_DECODE_GRID=$g > gpurun_out/lc/grid_$g.json 2>gpurun_out/lc/grid_$g.err || { echo "grid $g failed"; tail -3 gpurun_out/lc/grid_$g.err; exit 1; }
  echo "grid $g $(cat gpurun_out/lc/grid_$g.json)"
done
