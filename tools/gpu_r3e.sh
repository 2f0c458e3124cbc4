set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=tools/rb_mismatch.py
C30="--cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4"
timeout -k 10 120 python -u $R --cfg 27 --reps 3 > gpurun_out/r3e_asm27.log 2>&1 || exit $?
timeout -k 10 120 python -u $R $C30 --reps 3 > gpurun_out/r3e_asm30.log 2>&1 || exit $?
timeout -k 10 120 python -u $R $C30 --reps 2 --shape 64 64 3 1 1 32 56 > gpurun_out/r3e_asm30_l1.log 2>&1 || exit $?
timeout -k 10 120 python -u $R --cfg 27 --reps 2 --sentinel > gpurun_out/r3e_asm27s.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbnoasm.so timeout -k 10 120 python -u $R --cfg 27 --reps 3 > gpurun_out/r3e_noasm27.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbnoasm.so timeout -k 10 120 python -u $R $C30 --reps 3 > gpurun_out/r3e_noasm30.log 2>&1 || exit $?
cat gpurun_out/r3e_*.log | grep -v amdgpu.ids
