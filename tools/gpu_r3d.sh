set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py tests/test_gpu_mode_api.py tests/test_gpu_stem_pool.py > gpurun_out/r3d_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3d_all.log 2>&1
rc=$?
echo "all gpu rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r3d_bench.log 2>&1 || exit $?
tail -3 gpurun_out/r3d_new.log gpurun_out/r3d_all.log gpurun_out/r3d_bench.log
