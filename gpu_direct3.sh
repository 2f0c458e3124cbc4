set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/direct
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -u profile_engine.py --model mobilenet --batch 512 --reps 3 > $O/mbn_eng.log 2>&1
timeout -k 10 200 python -u profile_engine.py --depth 18 --batch 128 --reps 3 > $O/r18_eng.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --module-path 0 > $O/bench_r18.log 2>&1
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > $O/bench_mbn.log 2>&1
timeout -k 10 200 python -u tools/time_launch.py --model mobilenet --batch 512 --launch 1 3 --tiles 15 30 31 > $O/t_mbn3.log 2>&1
timeout -k 10 200 python -u tools/time_launch.py --depth 18 --batch 128 --launch 1 --tiles 15 30 31 > $O/t_r18_3.log 2>&1
