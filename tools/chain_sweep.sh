#!/bin/bash
# Residual-chain length sweep (QNN_ENGINE_MAX_LINKS 0..4; 0 = an fp32 map at every block output):
# images/s and in-graph contraction ms of the bench per setting.
# usage (on the box, from the repo root): bash tools/chain_sweep.sh OUTDIR "BENCH ARGS" [LINKS ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$1; A=$2; shift 2; mkdir -p $O
for L in ${@:-4 3 2 1 0}; do
  N=L${L}_$(echo $A | tr -d ' -')
  QNN_ENGINE_MAX_LINKS=$L timeout -k 10 300 python bench.py $A --steps 10 --warmup 3 --no-cpu-baseline --module-path 0 > $O/bench_$N.json 2> $O/bench_$N.err || { tail -5 $O/bench_$N.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('max_links', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['engine']['kernel_ms_per_forward'].get('qnn_qconv2d_fwd'))" $O/bench_$N.json "$L" "$A"
done
