#!/bin/bash
# usage: tools/gpurun_retry.sh <timeout> <command>  -- re-issues the gpurun call only while gpurun reports an
# infrastructure-side "transient" status (nothing ran, nothing charged); any real run, pass or fail, ends it
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  sleep 150
done
exit $rc
