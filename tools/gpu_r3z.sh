# wide LUT stores: full GPU suite + R18 sweep (product), then ablation sweeps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3z_tests.log 2>&1 || { tail -40 gpurun_out/r3z_tests.log; exit 1; }
tail -2 gpurun_out/r3z_tests.log
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --top 8 --json gpurun_out/r3z_sweep_r18.json > gpurun_out/r3z_sweep_r18.txt 2>&1 || exit $?
head -5 gpurun_out/r3z_sweep_r18.txt
bash tools/gpu_r3y.sh
