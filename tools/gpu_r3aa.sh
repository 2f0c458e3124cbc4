# two-pixel-tile K=576 configurations: parity tests + R18 sweep; R50 b256 sweep (headline tiles)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_parity.py tests/test_gpu_tiles.py tests/test_abi.py > gpurun_out/r3aa_tests.log 2>&1 || { tail -40 gpurun_out/r3aa_tests.log; exit 1; }
tail -2 gpurun_out/r3aa_tests.log
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --top 8 --json gpurun_out/r3aa_sweep_r18.json > gpurun_out/r3aa_sweep_r18.txt 2>&1 || exit $?
head -5 gpurun_out/r3aa_sweep_r18.txt
timeout -k 10 500 python -u tools/engine_sweep.py --depth 50 --batch 256 --top 8 --json gpurun_out/r3aa_sweep_r50.json > gpurun_out/r3aa_sweep_r50.txt 2>&1 || exit $?
grep -n "2304\]" gpurun_out/r3aa_sweep_r50.txt | head -4
