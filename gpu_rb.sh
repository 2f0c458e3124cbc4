# resident-band kernel: sweep (bitwise vs cfg 5 + timing), tile parity, full gpu tests, bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/sweep_tiles.py --reps 20 --only headline r50_l4 r50_l2 r50_l1 r50_3x3_s2 r18_l --cfgs 6 7 9 11 26 27 28 --json $O/rb_sweep.jsonl > $O/rb_sweep.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/rb_gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py > $O/rb_bench_default.log 2>&1
