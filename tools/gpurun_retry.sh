#!/bin/bash
# Re-submit a gpurun call ONLY when the infrastructure reports a transient
# failure (box not prepared / no slot); a command failure or GPU fault is
# never retried.  Usage: tools/gpurun_retry.sh <timeout> '<command>'
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[retry] transient infrastructure failure, attempt $i; sleeping 60s"
  sleep 60
done
exit 3
