# ablations of every configuration on every R18 b128 contraction (1 no loads, 2 no MFMA, 3 no epilogue)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 3 2 1; do
QNN_LIB=quantized.pytorch_amd/qnn/libqnn_hip_ablate$k.so timeout -k 10 300 python -u tools/engine_sweep.py --depth 18 --batch 128 --top 8 --json gpurun_out/r3y_sweep_r18_ab$k.json > gpurun_out/r3y_sweep_r18_ab$k.txt 2>&1 || exit $?
head -4 gpurun_out/r3y_sweep_r18_ab$k.txt
done
