set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export QNN_HALO=0
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for k in 0 1 3; do
  if [ $k = 0 ]; then unset QNN_LIB; else export QNN_LIB=$R/quantized.pytorch_amd/qnn/libqnn_hip_ablate$k.so; fi
  i=1
  for P in "$P1" "$P2"; do
    timeout -k 10 200 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/pmc_a$k/p$i -o p -- python3 $R/bench_layers.py --only headline_r50_l3_3x3_256 --reps 5 > $R/gpurun_out/pmc_a${k}_$i.log 2>&1
    i=$((i+1))
  done
done
