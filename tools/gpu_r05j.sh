# Round-5 call: kernel-trace profile of the long-code bench with the
# frame-interleaved decoder.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
QKD_ILV=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 tools/large_code_bench.py --qber 0.02 > $O/lc.log 2>&1 || { tail $O/lc.log; exit 1; }
tail -1 $O/lc.log
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r05j/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
