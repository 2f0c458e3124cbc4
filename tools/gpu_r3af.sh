# stem fused kernel: pooled rows per block 1/2/3 vs 4 (product) and its ablations, timed in place
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in libqnn_hip_sppr1.so libqnn_hip_sppr2.so libqnn_hip_sppr3.so; do
QNN_LIB=quantized.pytorch_amd/qnn/$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stem_pool.py > gpurun_out/r3af_tests_$L.log 2>&1 || { tail -30 gpurun_out/r3af_tests_$L.log; exit 1; }
echo "$L $(tail -1 gpurun_out/r3af_tests_$L.log)"
done
for L in libqnn_hip.so libqnn_hip_sppr1.so libqnn_hip_sppr2.so libqnn_hip_sppr3.so libqnn_hip_spabl1.so libqnn_hip_spabl2.so libqnn_hip_spabl3.so libqnn_hip_spabl4.so; do
QNN_LIB=quantized.pytorch_amd/qnn/$L timeout -k 10 200 python -u tools/time_ops.py --depth 18 --batch 128 --ops 1 >> gpurun_out/r3af_time.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/$L timeout -k 10 200 python -u tools/time_ops.py --depth 50 --batch 256 --ops 1 >> gpurun_out/r3af_time.log 2>&1 || exit $?
done
grep -v amdgpu gpurun_out/r3af_time.log
