# N = 70,000 (M = 35,000): the interleaved decoder with global target words
# against the split kernel (equality, then the long-code bench).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/ilv_equal_check.py 70000 1024 0.02 > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
grep equal $O/eq.log
for mode in d 0; do
  if [ $mode = d ]; then E=""; else E="QKD_ILV=0"; fi
  env $E timeout -k 10 300 python tools/large_code_bench.py --n 70000 --qber 0.02 > $O/lc_$mode.json 2> $O/lc_$mode.err || { tail -3 $O/lc_$mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/lc_$mode.json').read().strip().splitlines()[-1]);print('n=70000 ilv=$mode', round(d['ms_per_batch'],3), 'ms', round(d['gbit_s'],2), 'Gbit/s fer', d['fer'])"
done
