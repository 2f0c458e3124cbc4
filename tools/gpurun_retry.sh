# Run one gpurun call, re-trying only while no GPU box could be acquired (nothing ran, nothing was
# charged: gpurun exit 3, its infrastructure back-off notice, or a "transient" verdict in
# gpurun_out/.last_call.json).  Never re-runs a command that ran.
# usage: bash tools/gpurun_retry.sh LOG TIMEOUT 'COMMAND'
LOG=$1; TO=$2; CMD=$3
for a in 1 2 3 4 5 6 7 8 9 10 11 12; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ $rc -eq 3 ] || [ "$st" = "transient" ] || grep -q "no free box right now\|backing off after the last attempt" $LOG; then
    sleep 150; continue
  fi
  exit $rc
done
exit 3
