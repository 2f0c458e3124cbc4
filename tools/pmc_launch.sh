#!/bin/bash
# PMC passes over tools/time_launch.py (one launch of an engine plan under chosen tile
# configurations), one rocprofv3 run per counter group (gfx950 block limits), for comparing
# configurations of one layer by kernel name / dispatch in the counter CSVs.
# usage (on the box, from the repo root): bash tools/pmc_launch.sh OUTDIR 'TIME_LAUNCH ARGS'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; ARGS=$2
mkdir -p $O
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU"; do
  i=$((i + 1))
  echo "=== pass $i: $C $(date +%T)"
  timeout -s KILL 180 rocprofv3 --pmc $C -d $O/p$i -o run --output-format csv -- python3 tools/time_launch.py $ARGS > $O/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $O/p$i.log; exit 1; }
  tail -2 $O/p$i.log
done
