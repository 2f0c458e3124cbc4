# depthwise A/B: 8 channels/thread (product) vs 4 channels/thread at 3 or 4 waves/SIMD -- parity + MobileNet b512
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in libqnn_hip.so libqnn_hip_dw2a.so libqnn_hip_dw2b.so; do
export QNN_LIB=quantized.pytorch_amd/qnn/$L
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dwconv.py > gpurun_out/r3ae_tests_$L.log 2>&1 || { tail -30 gpurun_out/r3ae_tests_$L.log; exit 1; }
echo "$L $(tail -1 gpurun_out/r3ae_tests_$L.log)"
timeout -k 10 300 python -u bench.py --model mobilenet --batch 512 --no-cpu-baseline --module-path 0 > gpurun_out/r3ae_mbn_$L.json 2>> gpurun_out/r3ae.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r3ae_mbn_$L.json'));print('$L',d['value'],d['ms_per_step'],d['engine']['kernel_ms_per_forward'])"
done
