set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dwconv.py tests/test_gpu_engine.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/dw_tests.log 2>&1
timeout -k 10 300 python -u profile_engine.py --model mobilenet --batch 512 --reps 3 > $O/dw_prof_mbn.log 2>&1
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --steps 10 --warmup 3 --no-cpu-baseline > $O/dw_bench_mbn.log 2>&1
