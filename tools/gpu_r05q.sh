# The interleaved decoder against the split kernel across code lengths
# (random (3,6) codes, 4096 frames, QBER 0.02): QKD_ILV=0 / 1 forced, and the
# library's default choice.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
for n in 12000 16000 20000 24000 30000 40000 50000; do
  for mode in 0 1 d; do
    if [ $mode = d ]; then E=""; else E="QKD_ILV=$mode"; fi
    env $E timeout -k 10 200 python tools/large_code_bench.py --n $n --qber 0.02 > $O/n${n}_$mode.json 2> $O/n${n}_$mode.err \
      || { echo "n=$n mode=$mode failed: $(tail -1 $O/n${n}_$mode.err)"; continue; }
    python3 -c "import json;d=json.loads(open('$O/n${n}_$mode.json').read().strip().splitlines()[-1]);print('n=$n ilv=$mode', round(d['ms_per_batch'],3), 'ms', round(d['gbit_s'],2), 'Gbit/s', 'fer', d['fer'])"
  done
done
