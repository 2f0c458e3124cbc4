# round-3 re-entry baseline: full GPU suite, smoke, default bench (+ R50 b256, MobileNet b512)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3u_tests.log 2>&1 || { tail -30 gpurun_out/r3u_tests.log; exit 1; }
tail -2 gpurun_out/r3u_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3u_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3u_bench.json 2> gpurun_out/r3u_bench.err || exit $?
cat gpurun_out/r3u_bench.json
timeout -k 10 300 python -u bench.py --depth 50 --batch 256 --no-cpu-baseline --module-path 0 > gpurun_out/r3u_bench_r50.json 2>> gpurun_out/r3u_bench.err || exit $?
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > gpurun_out/r3u_bench_mbn.json 2>> gpurun_out/r3u_bench.err || exit $?
cut -c1-400 gpurun_out/r3u_bench_r50.json gpurun_out/r3u_bench_mbn.json
