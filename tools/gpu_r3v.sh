# every tile configuration of every contraction, in place: R18 b128 and R50 b256 (headline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --top 8 --json gpurun_out/r3v_sweep_r18.json > gpurun_out/r3v_sweep_r18.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/engine_sweep.py --depth 50 --batch 256 --top 8 --json gpurun_out/r3v_sweep_r50.json > gpurun_out/r3v_sweep_r50.txt 2>&1 || exit $?
tail -5 gpurun_out/r3v_sweep_r18.txt
