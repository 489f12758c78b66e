# PC sampling of the decoder (rocprofv3 beta): which instructions the waves sit
# on. Lists the box's PC-sampling configurations first; tries the stochastic
# (hardware, stall reasons) method, then host-trap. Each run has its own limit.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/pcs
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/list_avail.txt 2>&1
grep -i -B2 -A14 "pc_sampl\|pc sampl" $O/list_avail.txt | head -60
for m in stochastic host_trap; do
  u=cycles; iv=1048576
  [ $m = host_trap ] && { u=time; iv=100; }
  timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled 1 --pc-sampling-method $m --pc-sampling-unit $u \
    --pc-sampling-interval $iv --output-format csv -d $O/$m -o run -- python3 bench.py --steps 5 --warmup 1 \
    --no-cpu-baseline --no-variants --no-sweeps --no-e2e > $O/$m.log 2>&1
  echo "$m rc=$?"; tail -n 3 $O/$m.log
  ls -R $O/$m 2>/dev/null | head -20
done
