# vectorized s2d quantizer + back-to-back per-launch bench timing: parity, engine, bench (R18, R50, MobileNet)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_bench_parity.py tests/test_gpu_stem_pool.py > gpurun_out/r3ad_tests.log 2>&1 || { tail -40 gpurun_out/r3ad_tests.log; exit 1; }
tail -2 gpurun_out/r3ad_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3ad_bench.json 2> gpurun_out/r3ad_bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r3ad_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac'],d['engine'])"
timeout -k 10 300 python -u bench.py --depth 50 --batch 256 --no-cpu-baseline --module-path 0 > gpurun_out/r3ad_bench_r50.json 2>> gpurun_out/r3ad_bench.err || exit $?
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > gpurun_out/r3ad_bench_mbn.json 2>> gpurun_out/r3ad_bench.err || exit $?
for f in r50 mbn; do python -c "import json;d=json.load(open('gpurun_out/r3ad_bench_$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d['engine']['kernel_ms_per_forward'])"; done
