# Kernel timelines of the long-code bench with the follower on / off
# (profiles/r05_ilv_follower_timeline.jsonl). The follower launch was measured
# slower and removed: QKD_ILV_FOLLOW is no longer read, so
# both runs of this script now time the same build.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for f in 1 0; do
  QKD_ILV_FOLLOW=$f timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$f -o run -- \
    python3 tools/large_code_bench.py --qber 0.02 > $O/lc_$f.json 2> $O/lc_$f.err || { tail $O/lc_$f.err; exit 1; }
done
find $O -name "*kernel_trace.csv" | head
