# round-2 verification and evidence: gpu tests, smoke, benches (R18 b128 default, R50 b256,
# MobileNet b512), rocprofv3 kernel stats of the default bench, per-launch rocprof tables
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/f_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/f_smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/f_bench_default.log 2>&1
timeout -k 10 300 python -u bench.py --depth 50 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > $O/f_bench_r50.log 2>&1
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --steps 10 --warmup 3 --no-cpu-baseline > $O/f_bench_mbn.log 2>&1
timeout -k 10 300 python -u bench_layers.py --only headline > $O/f_layers_headline.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f_rp_r18 -o rp -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --module-path 0 > $O/f_rp_r18.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/f_lt_r50 -o run -- python3 $R/tools/layer_table.py run --depth 50 --batch 256 --meta $O/f_lt_r50_meta.json > $O/f_lt_r50.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/f_lt_r18 -o run -- python3 $R/tools/layer_table.py run --depth 18 --batch 128 --meta $O/f_lt_r18_meta.json > $O/f_lt_r18.log 2>&1
