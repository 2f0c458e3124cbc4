set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/pmc_r18
mkdir -p $D
export TMPDIR=/tmp
A="--model resnet --depth 18 --batch 128 --fwd 2 --eager"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $D/p1 -o run -- python3 tools/layer_table.py run $A --meta $D/meta.json > $D/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $D/p2 -o run -- python3 tools/layer_table.py run $A --meta $D/meta2.json > $D/p2.log 2>&1 || exit $?
python3 tools/pmc_table.py $D/meta.json $D/p1 $D/p2 --json $D/pmc.json
