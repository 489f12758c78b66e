# Round-5 measurement call: counter list, LDS bank microbenchmark (+PMC), the
# GPU tests touched this round, A/B of the experiment builds in exp_libs/ against
# the in-tree library (tools/gpu_ab.sh), phase shares, then VALU-mix PMC passes.
# Outputs under gpurun_out/r05b. Every GPU step has its own time limit and any
# failure ends the script.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 100); do sleep 30; date >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 120 ./tools/mb/issue_mb > $O/issue_mb.txt 2>&1 || { cat $O/issue_mb.txt; exit 1; }
grep "waves/SIMD  4.0" $O/issue_mb.txt
timeout -k 10 60 ./tools/mb/lds_bank_mb tools/mb/lds_stream.bin > $O/lds_mb.txt 2>&1 || { cat $O/lds_mb.txt; exit 1; }
cat $O/lds_mb.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/lds_pmc -o run -- ./tools/mb/lds_bank_mb tools/mb/lds_stream.bin > $O/lds_pmc.log 2>&1 || { tail $O/lds_pmc.log; exit 1; }
python3 - $O/lds_pmc <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in v.items():
    print(k, {n: int(x) for n, x in c.items()}, "conflict/idx=%.3f" % (c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_LDS_IDX_ACTIVE"])))
PY
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py tests/test_large_codes.py tests/test_spec.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
REPS=${REPS:-3} bash tools/gpu_ab.sh > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
QKD_PHASE_TIMING=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-sweeps --no-variants --no-e2e --steps 20 > $O/phase.json 2> $O/phase.err || { tail $O/phase.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/phase.json').read().strip().splitlines()[-1]);print('phase', {k: round(v,4) for k,v in d['phase_share'].items()})"
