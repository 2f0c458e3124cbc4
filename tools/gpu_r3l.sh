set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --json gpurun_out/r3l_sweep_r18.json > gpurun_out/r3l_sweep_r18.txt 2>&1 || exit $?
cat gpurun_out/r3l_sweep_r18.txt | grep -v amdgpu
