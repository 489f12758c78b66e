# Target syndrome words in global memory (the interleaved decoder's LDS then
# fits M up to ~36,000): parity, equality with the split kernel at N = 50,000
# and 60,000, and the long-code bench against the previous build (base0).
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_large_codes.py -q -x -k "interleaved" --timeout 200 \
  --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -n 1 $O/parity.log
for n in 50000 60000; do
  timeout -k 10 300 python tools/ilv_equal_check.py $n 1024 0.02 > $O/eq_$n.log 2>&1 || { echo "eq $n failed"; tail -5 $O/eq_$n.log; exit 1; }
  cat $O/eq_$n.log
done
for r in 1; do
  for n in 40000 50000 60000; do
    for l in new base0; do
      if [ $l = new ]; then L=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; else L=exp_libs/base0/libqkd_ldpc_amd.so; fi
      QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$L timeout -k 10 200 python tools/large_code_bench.py --n $n --qber 0.02 \
        > $O/lc_${n}_$l.json 2> $O/lc_${n}_$l.err || { echo "n=$n $l failed: $(tail -1 $O/lc_${n}_$l.err)"; continue; }
      python3 -c "import json;d=json.loads(open('$O/lc_${n}_$l.json').read().strip().splitlines()[-1]);print('n=$n $l', round(d['ms_per_batch'],3), 'ms', round(d['gbit_s'],2), 'Gbit/s fer', d['fer'])"
    done
  done
done
