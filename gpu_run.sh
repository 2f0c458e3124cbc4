set -e
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
for c in 6 7 3; do
  QNN_CONV_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_cfg$c.log 2>&1
done
timeout -k 10 200 python -u profile_engine.py > gpurun_out/prof_engine.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
