#!/bin/bash
# The no-packed-FP32 policy's cost: the three benches with the product library and with the
# packed-FP32 diagnostic build (make -C quantized.pytorch_amd qnn/libqnn_hip_pk.so), alternating.
# usage (on the box, from the repo root): bash tools/pk_compare.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$1; mkdir -p $O
for rep in 1 2; do
  for V in "" pk; do
    L=$PWD/quantized.pytorch_amd/qnn/libqnn_hip${V:+_$V}.so
    for A in "--depth 18 --batch 128" "--depth 50 --batch 256" "--model mobilenet --batch 512"; do
      N=${V:-default}_$(echo $A | tr -d ' -')_$rep
      QNN_LIB=$L timeout -k 10 300 python bench.py $A --steps 20 --warmup 5 --no-cpu-baseline --module-path 0 > $O/$N.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['engine']['kernel_ms_per_forward'])" $O/$N.json $N
    done
  done
done
