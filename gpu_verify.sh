# verification: gpu tests, smoke, default bench, rocprofv3 kernel stats of the bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/v_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/v_smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/v_bench_default.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v_rp_r18 -o rp -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --module-path 0 > $O/v_rp_r18.log 2>&1
