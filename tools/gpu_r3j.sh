set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=tools/rb_mismatch.py
C30="--cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4"
timeout -k 10 120 python -u $R $C30 --reps 4 --shape 128 128 3 1 1 256 28 > gpurun_out/r3j_mm.log 2>&1 || exit $?
timeout -k 10 120 python -u $R $C30 --reps 4 >> gpurun_out/r3j_mm.log 2>&1 || exit $?
timeout -k 10 120 python -u $R --cfg 27 --reps 4 >> gpurun_out/r3j_mm.log 2>&1 || exit $?
grep -h "rep \|config" gpurun_out/r3j_mm.log
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3j_all.log 2>&1
rc=$?
tail -8 gpurun_out/r3j_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r3j_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3j_bench.log | cut -c1-1500
