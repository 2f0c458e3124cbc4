# GPU session: tile parity (all configs incl. qconv16), per-layer tile sweep
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread -k "mode0" > gpurun_out/gpu_tiles_m0.log 2>&1 || { tail -40 gpurun_out/gpu_tiles_m0.log; exit 1; }
timeout -k 10 400 python -u tools/sweep_tiles.py --reps 10 --json gpurun_out/sweep.jsonl > gpurun_out/sweep.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tiles.log 2>&1 || { tail -40 gpurun_out/gpu_tiles.log; exit 1; }
