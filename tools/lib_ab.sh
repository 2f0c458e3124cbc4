#!/bin/bash
# A/B of diagnostic library builds on one bench: in-graph ms per forward of one launch kind.
# usage (on the box, from the repo root): bash tools/lib_ab.sh OUTDIR KIND "BENCH ARGS" SUFFIX...
#   SUFFIX "-" = the product library; else quantized.pytorch_amd/qnn/libqnn_hip_SUFFIX.so
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$1; K=$2; A=$3; shift 3; mkdir -p $O
for V in "$@"; do
  [ "$V" = "-" ] && L=quantized.pytorch_amd/qnn/libqnn_hip.so || L=quantized.pytorch_amd/qnn/libqnn_hip_$V.so
  N=${V}_$(echo $A | tr -d ' -')
  QNN_LIB=$PWD/$L timeout -k 10 300 python bench.py $A --steps 10 --warmup 3 --no-cpu-baseline --module-path 0 > $O/bench_$N.json 2> $O/bench_$N.err || { tail -5 $O/bench_$N.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['engine']['kernel_ms_per_forward'].get(sys.argv[4]))" $O/bench_$N.json "$V" "$A" "$K"
done
