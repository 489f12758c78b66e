# Round-5 probe: counter list, LDS bank microbenchmark (+ its PMC pass), the
# multi-GPU tests and a headline bench line. Outputs under gpurun_out/r05a.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || echo "list rc=$?"
timeout -k 10 60 ./tools/mb/lds_bank_mb tools/mb/lds_stream.bin > $O/lds_mb.txt 2>&1 || { cat $O/lds_mb.txt; exit 1; }
cat $O/lds_mb.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/lds_pmc -o run -- ./tools/mb/lds_bank_mb tools/mb/lds_stream.bin > $O/lds_pmc.log 2>&1 || { tail $O/lds_pmc.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py tests/test_large_codes.py tests/test_spec.py -x -v --timeout 200 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 1; }
tail -3 $O/pytest_dist.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sweeps --no-variants --steps 20 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python tools/bench_brief.py $O/bench.json
