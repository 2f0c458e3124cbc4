# K=576 direct-fragment configurations: full GPU suite, R18 b128 sweep, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3w_tests.log 2>&1 || { tail -40 gpurun_out/r3w_tests.log; exit 1; }
tail -2 gpurun_out/r3w_tests.log
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --top 6 --json gpurun_out/r3w_sweep_r18.json > gpurun_out/r3w_sweep_r18.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err || exit $?
cut -c1-300 gpurun_out/r3w_bench.json
