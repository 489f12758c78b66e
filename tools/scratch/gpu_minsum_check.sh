# GPU check of the min-sum variants: their bit-exact tests, then the FER sweep of
# plain and self-corrected min-sum over scales at config 3's hardest points.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_variants.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_minsum.log 2>&1; rc=$?
tail -n 3 gpurun_out/pytest_minsum.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/minsum_sweep.py --trials 100000 --qbers ${QBERS:-0.07,0.08} --scales ${SCALES:-0.75,0.8125,0.875,0.9375} \
  --offsets 0 --self-correct 0,1 > gpurun_out/minsum_sc_sweep.jsonl 2> gpurun_out/minsum_sc_sweep.err || exit $?
python -c "
import json
for l in open('gpurun_out/minsum_sc_sweep.jsonl'):
    d=json.loads(l); print(d['variant'], d['scale'], d.get('self_correct'), round(d['qber'],3), d['fer'], round(d['mean_it'],2), round(d['ms'],1))"
