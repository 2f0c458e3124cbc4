set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread -k "mode0" > gpurun_out/gpu_tiles_m0.log 2>&1 || { tail -40 gpurun_out/gpu_tiles_m0.log; exit 1; }
timeout -k 10 400 python -u tools/sweep_tiles.py --reps 10 --json gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1
QNN_LIB=$PWD/quantized.pytorch_amd/qnn/libqnn_hip_ablate3.so timeout -k 10 300 python -u tools/sweep_tiles.py --reps 10 --json gpurun_out/sweep_ablate3.jsonl > gpurun_out/sweep_ablate3.log 2>&1
