set -e
mkdir -p gpurun_out
export QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_stamp.so
timeout -k 10 200 python -u tools/stamps.py --engine 1 3 4 7 9 10 14 15 19 20 > gpurun_out/stamps_engine.log 2>&1
for c in 0 6 9 7; do QNN_CONV_CFG=$c timeout -k 10 100 python -u tools/stamps.py --layer headline > gpurun_out/stamps_head_c$c.log 2>&1; done
unset QNN_LIB
for c in 0 6 9 1 7; do QNN_CONV_CFG=$c timeout -k 10 100 python -u bench_layers.py --only headline r18_l3 > gpurun_out/layers_c$c.log 2>&1; done
