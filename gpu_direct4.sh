set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/direct
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread -k "30 or 31 or 32" > $O/tiles4.log 2>&1
timeout -k 10 200 python -u tools/time_launch.py --model mobilenet --batch 512 --launch 5 7 9 11 --tiles 11 31 32 > $O/t_mbn4.log 2>&1
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > $O/bench_mbn4.log 2>&1
timeout -k 10 200 python -u profile_engine.py --model mobilenet --batch 512 --reps 3 > $O/mbn_eng4.log 2>&1
