set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=tools/rb_mismatch.py
C30="--cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4"
export QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_pkam.so
timeout -k 10 120 python -u $R $C30 --reps 4 --shape 128 128 3 1 1 256 28 > gpurun_out/r3s_mm.log 2>&1 || exit $?
timeout -k 10 120 python -u $R $C30 --reps 4 >> gpurun_out/r3s_mm.log 2>&1 || exit $?
timeout -k 10 120 python -u $R --cfg 27 --reps 4 >> gpurun_out/r3s_mm.log 2>&1 || exit $?
grep -h "rep \|config" gpurun_out/r3s_mm.log
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py tests/test_gpu_tiles.py -k "bench_batch or natural" > gpurun_out/r3s_tests.log 2>&1
tail -3 gpurun_out/r3s_tests.log
timeout -k 10 200 python -u tools/time_ops.py --depth 18 --batch 128 --ops 1 3 5 > gpurun_out/r3s_time.log 2>&1 || exit $?
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip.so timeout -k 10 200 python -u tools/time_ops.py --depth 18 --batch 128 --ops 1 3 5 >> gpurun_out/r3s_time.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r3s_time.log
