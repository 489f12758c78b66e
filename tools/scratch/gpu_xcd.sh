set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/xcd; mkdir -p $O
PARITY_K=config2_every_cap REPS=3 bash tools/gpu_ab.sh || exit 1
for l in base xcd; do
  lib=qkd_ldpc_amd/lib/libqkd_ldpc_amd.so; [ $l = base ] || lib=exp_libs/$l/libqkd_ldpc_amd.so
  for c in WRITE_SIZE FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/$l -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-e2e --no-sweeps > $O/$l.log 2>&1 || exit 1
    python3 - $O/$l <<'PY'
import csv,glob,sys,collections
c=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/run_counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if "decode_split" in r["Kernel_Name"]: c[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1], {k: "%.4g" % (sum(v)/len(v)) for k,v in c.items()})
PY
    rm -rf $O/$l
  done
done
