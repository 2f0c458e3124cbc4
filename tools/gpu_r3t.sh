set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -v --timeout 60 --timeout-method thread tests/test_gpu_comm.py > gpurun_out/r3t_comm.log 2>&1
tail -3 gpurun_out/r3t_comm.log
bash tools/gpu_prof.sh mbn_b512 mobilenet 18 512 || exit $?
