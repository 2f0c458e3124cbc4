set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python profile_engine.py > gpurun_out/prof_v5.log 2>&1
export QNN_LIB=$PWD/quantized.pytorch_amd/qnn/libqnn_hip_stamp.so
timeout -k 10 300 python tools/stamps.py --engine 1 3 4 7 9 10 15 16 20 > gpurun_out/stamps_engine.log 2>&1
