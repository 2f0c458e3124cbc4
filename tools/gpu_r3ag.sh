# training-side quantization tests (§8(f4)) + the whole GPU suite, then the stem variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py > gpurun_out/r3ag_train.log 2>&1 || { tail -40 gpurun_out/r3ag_train.log; exit 1; }
tail -2 gpurun_out/r3ag_train.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3ag_tests.log 2>&1 || { tail -40 gpurun_out/r3ag_tests.log; exit 1; }
tail -2 gpurun_out/r3ag_tests.log
bash tools/gpu_r3af.sh
