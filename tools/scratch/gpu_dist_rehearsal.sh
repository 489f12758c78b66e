# Multi-rank rehearsal of bench.py on one GPU: two ranks over gloo sharing the
# device (the RCCL collective itself needs one GPU per rank).
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
QKD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/dist2.log 2>&1 || { tail -n 30 gpurun_out/dist2.log; exit 1; }
grep '^{' gpurun_out/dist2.log | tail -1 | cut -c1-600
