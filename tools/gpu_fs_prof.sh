set -u
cd /root/repo
export TMPDIR=/tmp
for l in new old; do
  lib=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; [ $l = old ] && lib=exp_libs/r06c_old/libqkd_ldpc_amd.so
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fs_$l -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-variants --no-sweeps > gpurun_out/fs_$l.log 2>&1 || { tail -5 gpurun_out/fs_$l.log; exit 3; }
  python3 tools/prof_summary.py gpurun_out/fs_$l gpurun_out/fs_$l.json || exit 4
  python3 -c "
import json; d=json.load(open('gpurun_out/fs_$l.json'))
for r in d['kernels'][:8]: print('$l', round(r['warm_avg_ms']*1000,1), 'us', r['warm_dispatches'], r['kernel'][:70])"
done
