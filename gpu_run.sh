set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --module-path 0 > gpurun_out/bench_r18.log 2>&1
timeout -k 10 300 python -u bench.py --depth 50 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline --module-path 0 > gpurun_out/bench_r50.log 2>&1
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --steps 10 --warmup 3 --no-cpu-baseline --module-path 0 > gpurun_out/bench_mbn.log 2>&1
timeout -k 10 200 python -u profile_engine.py --depth 18 --batch 128 --reps 3 > gpurun_out/prof_r18.log 2>&1
