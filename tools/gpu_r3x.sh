# K=576 direct-fragment: no-prefetch variant; direct parity tests + R18 b128 sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_parity.py tests/test_gpu_tiles.py > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -2 gpurun_out/r3x_tests.log
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --top 8 --json gpurun_out/r3x_sweep_r18.json > gpurun_out/r3x_sweep_r18.txt 2>&1 || exit $?
head -6 gpurun_out/r3x_sweep_r18.txt
