set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "" sppr1 sppr2 sppr3; do
  L=quantized.pytorch_amd/qnn/libqnn_hip${v:+_$v}.so
  QNN_LIB=$L timeout -k 10 200 python -u tools/time_ops.py --depth 18 --batch 128 --ops 0 1 >> gpurun_out/r3o.log 2>&1 || exit $?
done
grep -v amdgpu gpurun_out/r3o.log
