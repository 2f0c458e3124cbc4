set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 27 --reps 2 --sentinel > gpurun_out/r3c_asm27s.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbswait.so timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 27 --reps 3 > gpurun_out/r3c_swait27.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_rbswait.so timeout -k 10 120 python -u tools/rb_mismatch.py --cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4 --reps 3 > gpurun_out/r3c_swait30.log 2>&1 || exit $?
cat gpurun_out/r3c_*.log | grep -v amdgpu.ids | grep -v "^  [a-z]"
