set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 27 --reps 3 > gpurun_out/r3b_asm27.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4 --reps 2 > gpurun_out/r3b_asm30.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbnoasm.so timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 27 --reps 3 > gpurun_out/r3b_noasm27.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbnoasm.so timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4 --reps 2 > gpurun_out/r3b_noasm30.log 2>&1 || exit $?
cat gpurun_out/r3b_*.log | grep -v amdgpu.ids
