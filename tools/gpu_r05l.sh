# Round-5 call: hand-off counts and the exact-kernel hand-off variant.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
for fb in spec exact; do
  QKD_ILV=1 QKD_ILV_FB=$fb QKD_ILV_STATS=1 timeout -k 10 200 python tools/large_code_bench.py --qber 0.02 > $O/lc_$fb.json 2> $O/lc_$fb.err || { tail $O/lc_$fb.err; exit 1; }
  sort $O/lc_$fb.err | uniq -c | head -5; cut -c1-120 $O/lc_$fb.json
done
QKD_ILV=1 QKD_ILV_FB=exact timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 tools/large_code_bench.py --qber 0.02 > $O/lc.log 2>&1 || { tail $O/lc.log; exit 1; }
python3 tools/prof_summary.py $O/trace $O/kernel_summary.json | head -4
