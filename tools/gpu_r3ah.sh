# round-3 closing evidence: training tests, full GPU suite, smoke, default bench, rocprof stats of
# the bench command itself; then the stem variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py > gpurun_out/r3ah_train.log 2>&1 || { tail -40 gpurun_out/r3ah_train.log; exit 1; }
tail -2 gpurun_out/r3ah_train.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3ah_tests.log 2>&1 || { tail -40 gpurun_out/r3ah_tests.log; exit 1; }
tail -2 gpurun_out/r3ah_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ah_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3ah_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3ah_bench.json 2> gpurun_out/r3ah_bench.err || exit $?
cut -c1-200 gpurun_out/r3ah_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 20 --no-cpu-baseline --module-path 0 > gpurun_out/r3ah_bench_rocprof.log 2>&1 || exit $?
timeout -k 10 300 python -u bench_layers.py --only headline r50_l4 > gpurun_out/r3ah_headline.jsonl 2>> gpurun_out/r3ah_bench.err || exit $?
cut -c1-300 gpurun_out/r3ah_headline.jsonl
