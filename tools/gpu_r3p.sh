set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/time_ops.py --depth 18 --batch 128 --ops 0 1 > gpurun_out/r3p.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_stem_pool.py >> gpurun_out/r3p.log 2>&1
grep -v amdgpu gpurun_out/r3p.log | tail -5
