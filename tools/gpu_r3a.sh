set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py tests/test_gpu_mode_api.py > gpurun_out/r3a_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3a_all.log 2>&1
echo "all gpu rc=$?"
tail -5 gpurun_out/r3a_new.log gpurun_out/r3a_all.log
