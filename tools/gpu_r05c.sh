# A/B of exp_libs/ builds against the in-tree library (tools/gpu_ab.sh), with
# extra LIBS entries from the caller (e.g. "base@QKD_SPEC_POLICY=always").
# Outputs under gpurun_out/r05c.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 100); do sleep 30; date >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
REPS=${REPS:-3} LIBS="${LIBS:-}" bash tools/gpu_ab.sh > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
