set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=tools/rb_mismatch.py
C30="--cfg 30 --bm 128 --bn 128 --wgm 4 --wgn 2 --tm 2 --tn 4"
for v in "" rbnopk rbnoasm rbnoasmnopk; do
  L=quantized.pytorch_amd/qnn/libqnn_hip${v:+_$v}.so
  echo "=== $L" >> gpurun_out/r3h.log
  QNN_LIB=$L timeout -k 10 120 python -u $R $C30 --reps 3 --shape 128 128 3 1 1 256 28 >> gpurun_out/r3h.log 2>&1 || exit $?
  QNN_LIB=$L timeout -k 10 120 python -u $R $C30 --reps 3 >> gpurun_out/r3h.log 2>&1 || exit $?
  QNN_LIB=$L timeout -k 10 120 python -u $R --cfg 27 --reps 3 >> gpurun_out/r3h.log 2>&1 || exit $?
done
grep -h "===\|rep \|config" gpurun_out/r3h.log
