#!/bin/bash
# Named GPU measurements (run on the GPU box): tools/gpu_presets.sh <preset> [args]
# Each GPU step has its own time limit; a failure ends the script. Outputs under
# gpurun_out/<preset>. Library options go through --debug-opt (the library reads
# no environment variable, include/qkd_ldpc.h qkd_debug_set_option).
#   lengths [N...]     the interleaved decoder (QKD_ILV=1), the split kernel
#                      (QKD_ILV=0) and the default choice across random (3,6)
#                      code lengths, 4096 frames, QBER 0.02 (profiles/r05_ilv_length_sweep.txt)
#   long_equal [N...]  interleaved == split on 1024 frames, then the long-code
#                      bench (default choice and QKD_ILV=0) at each N
#   ilv_phases         interleaved phase shares: a diagnostic build with
#                      -DQKD_ILV_PHASES in exp_libs/ilvph (tools/ab_build.sh),
#                      N = 40,000, QBER 0.02 / 0.03 (profiles/r05_ilv_phases.txt)
#   e2e_timeline       kernel timeline of the decode-only and end-to-end steps
#                      (tools/e2e_timeline.py; profiles/r05_e2e_timeline.txt)
#   variants [V...]    per-variant phase shares and one PMC pass (core counters)
#   minsum             the min-sum / binary32 parity tests, then each variant's bench
set -u
cd "$(dirname "$0")/.."
P=${1:?preset}; shift
O=gpurun_out/$P
mkdir -p $O
export TMPDIR=/tmp
lc() {  # lc <tag> <bench args...>: one long-code bench run, one summary line
  local tag=$1; shift
  timeout -k 10 300 python tools/large_code_bench.py "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed: $(tail -1 $O/$tag.err)"; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);print('$tag', round(d['ms_per_batch'],3), 'ms', round(d['gbit_s'],2), 'Gbit/s fer', d['fer'])"
}
case $P in
lengths)
  for n in ${@:-12000 16000 20000 24000 30000 40000 50000}; do
    lc n${n}_ilv1 --n $n --qber 0.02 --debug-opt QKD_ILV=1 || true
    lc n${n}_ilv0 --n $n --qber 0.02 --debug-opt QKD_ILV=0 || true
    lc n${n}_default --n $n --qber 0.02 || true
  done ;;
long_equal)
  for n in ${@:-50000 60000 70000}; do
    timeout -k 10 300 python tools/ilv_equal_check.py $n 1024 0.02 > $O/eq_$n.log 2>&1 || { tail -5 $O/eq_$n.log; exit 1; }
    grep equal $O/eq_$n.log
    lc n${n}_default --n $n --qber 0.02 || exit 1
    lc n${n}_ilv0 --n $n --qber 0.02 --debug-opt QKD_ILV=0 || exit 1
  done ;;
ilv_phases)
  for q in 0.02 0.03; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=exp_libs/ilvph/libqkd_ldpc_amd.so timeout -k 10 200 \
      python tools/large_code_bench.py --qber $q --phase-timing > $O/ph_$q.json 2> $O/ph_$q.err || { tail $O/ph_$q.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/ph_$q.json').read().strip().splitlines()[-1]);print('q=$q', round(d['ms_per_batch'],3), d['phase_share'][:4], d['phase_cycles'][:4])"
  done ;;
e2e_timeline)
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 tools/e2e_timeline.py \
    > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
  python3 tools/e2e_timeline.py --summarise $O/p/run_kernel_trace.csv ;;
variants)
  for v in ${@:-minsum sp_f32}; do
    timeout -k 10 120 python bench.py --variant $v --phase-timing --no-cpu-baseline --no-variants --no-sweeps --no-e2e \
      --steps 10 > $O/phase_$v.json 2> $O/phase_$v.err || { tail $O/phase_$v.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$O/phase_$v.json').read().strip().splitlines()[-1])
print('$v', round(d['roofline']['kernel_ms'], 4), 'ms', {k: round(x, 3) for k, x in d.get('phase_share', {}).items()})"
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
      SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --variant $v \
      --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-e2e --no-sweeps > $O/pmc_$v.log 2>&1 \
      || { echo "pmc $v failed"; tail $O/pmc_$v.log; exit 1; }
    python3 - $O/pmc_$v $v <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "decode" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(x) / len(x)) for k, x in v.items()})
PY
  done ;;
minsum)
  timeout -k 10 600 python -u -m pytest tests/test_variants.py tests/test_spec.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "minsum or packed_phi or sp_f32" > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log
  [ $rc -eq 0 ] || { grep -B3 -A30 "Error\|FAILED\|assert" $O/pytest.log | head -60; exit $rc; }
  for v in minsum minsum_sc sp_f32; do
    timeout -k 10 120 python bench.py --variant $v --no-cpu-baseline --no-variants --no-sweeps --no-e2e --steps 20 \
      > $O/bench_$v.json 2> $O/bench_$v.err || { tail $O/bench_$v.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1])
print('$v', 'step', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'mean it', d['mean_iterations'])"
  done ;;
*) echo "unknown preset $P"; exit 2 ;;
esac
