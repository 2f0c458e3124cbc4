set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread -k "mode0" > gpurun_out/gpu_tiles_m0.log 2>&1 || { tail -40 gpurun_out/gpu_tiles_m0.log; exit 1; }
timeout -k 10 400 python -u tools/sweep_tiles.py --reps 10 --only headline r50_l4 r18_l1 r18_l2 r18_l3 r18_l4 stem --json gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1
for a in 3 2; do
QNN_LIB=$PWD/quantized.pytorch_amd/qnn/libqnn_hip_ablate$a.so timeout -k 10 300 python -u tools/sweep_tiles.py --reps 10 --only headline r18_l1 r18_l4 --json gpurun_out/sweep_ablate$a.jsonl > gpurun_out/sweep_ablate$a.log 2>&1
done
