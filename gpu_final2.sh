set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > $O/bench_mbn.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
