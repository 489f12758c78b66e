# Phase shares of the interleaved decoder (diagnostic build -DQKD_ILV_PHASES,
# exp_libs/ilvph) on the long-code bench, N = 40,000, QBER 0.02 and 0.03.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
for q in 0.02 0.03; do
  QKD_PHASE_TIMING=1 QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=exp_libs/ilvph/libqkd_ldpc_amd.so timeout -k 10 200 \
    python tools/large_code_bench.py --qber $q > $O/ph_$q.json 2> $O/ph_$q.err || { tail $O/ph_$q.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/ph_$q.json').read().strip().splitlines()[-1]);print('q=$q', round(d['ms_per_batch'],3), d['phase_share'][:4], d['phase_cycles'][:4])"
done
