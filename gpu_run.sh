# GPU session script: tile-parity tests, the full gpu suite, default bench
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_tiles.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tiles.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_tiles.py > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r18.log 2>&1
