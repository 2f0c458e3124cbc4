#!/bin/bash
# Stem max-pool ablations (make -C quantized.pytorch_amd spablate): in-graph stem time of the
# ResNet-18 b128 and ResNet-50 b256 benches with each ablated library (QNN_SP_ABLATE: 1 no MFMA,
# 2 no tile epilogue, 3 no pooling, 4 no band DMA).  Timing only: ablated outputs are wrong.
# usage (on the box, from the repo root): bash tools/sp_ablate.sh OUTDIR [SUFFIX ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$1; shift; mkdir -p $O
VS=${@:-"- spabl1 spabl2 spabl3 spabl4"}
for V in $VS; do
  [ "$V" = "-" ] && L=quantized.pytorch_amd/qnn/libqnn_hip.so || L=quantized.pytorch_amd/qnn/libqnn_hip_$V.so
  for A in "--depth 18 --batch 128" "--depth 50 --batch 256"; do
    N=${V}_$(echo $A | tr -d ' -')
    QNN_LIB=$PWD/$L timeout -k 10 300 python bench.py $A --steps 10 --warmup 3 --no-cpu-baseline --module-path 0 > $O/bench_$N.json 2> $O/bench_$N.err || { tail -5 $O/bench_$N.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['engine']['kernel_ms_per_forward']['qnn_qconv2d_maxpool_fwd'])" $O/bench_$N.json "$V" "$A"
  done
done
