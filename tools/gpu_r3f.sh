set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=tools/rb_mismatch.py
C30="--cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4"
timeout -k 10 120 python -u $R --cfg 27 --reps 3 > gpurun_out/r3f_asm27.log 2>&1 || exit $?
timeout -k 10 120 python -u $R $C30 --reps 3 > gpurun_out/r3f_asm30.log 2>&1 || exit $?
timeout -k 10 120 python -u $R $C30 --reps 2 --shape 64 64 3 1 1 32 56 > gpurun_out/r3f_asm30_l1.log 2>&1 || exit $?
grep -h "rep \|library" gpurun_out/r3f_*.log
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3f_all.log 2>&1
rc=$?
tail -12 gpurun_out/r3f_all.log
exit $rc
