#!/bin/bash
# Stem max-pool variants (make -C quantized.pytorch_amd spdiag): each variant library's stem tests,
# then the in-graph stem time of the ResNet-18 b128 and ResNet-50 b256 benches.
# usage (on the box, from the repo root): bash tools/sp_variants.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$1; mkdir -p $O
for V in "" sp1 sp2 sp3; do
  L=quantized.pytorch_amd/qnn/libqnn_hip${V:+_$V}.so
  echo "=== variant ${V:-default} $(date +%T)"
  QNN_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stem_pool.py > $O/test_${V:-default}.log 2>&1 || { tail -5 $O/test_${V:-default}.log; exit 1; }
  tail -1 $O/test_${V:-default}.log
  for A in "--depth 18 --batch 128" "--depth 50 --batch 256"; do
    QNN_LIB=$PWD/$L timeout -k 10 300 python bench.py $A --steps 10 --warmup 3 --no-cpu-baseline --module-path 0 > $O/bench_${V:-default}_$(echo $A | tr -d ' -').json 2> $O/bench_err.log || { tail -5 $O/bench_err.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['engine']['kernel_ms_per_forward']['qnn_qconv2d_maxpool_fwd'])" $O/bench_${V:-default}_$(echo $A | tr -d ' -').json "$A"
  done
done
