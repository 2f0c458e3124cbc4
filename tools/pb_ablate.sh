# usage (on the box): bash tools/pb_ablate.sh OUT   -- persistent-band ablations (make pbablate) on ResNet-18 b128
# layer-1 launches 3 (code-table epilogue) and 4 (general chain); configuration 11 is the unaffected control
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
for L in "" 1 2 3 4 5; do
  LIB=""; [ -n "$L" ] && LIB=$PWD/quantized.pytorch_amd/qnn/libqnn_hip_pbabl$L.so
  echo "== ablation ${L:-none}" | tee -a $O/ablate.txt
  QNN_LIB=$LIB timeout -k 10 300 python -u tools/time_launch.py --launch 3 4 --tiles 11 45 46 47 --reps 20 2>&1 | grep -v amdgpu.ids | tee -a $O/ablate.txt || exit $?
done
