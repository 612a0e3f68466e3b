#!/bin/bash
# Run one gpurun call; re-submit only when the infrastructure reports a transient failure
# before the command started (status "transient" / exit 3: nothing ran, nothing charged).
# Usage: tools/gpucall.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpucall.out 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = "3" ] || [ "$st" = "transient" ]; then
    echo "[gpucall] transient (attempt $attempt), retrying in 40s" >&2; sleep 40; continue
  fi
  tail -4 /tmp/gpucall.out
  exit $rc
done
tail -4 /tmp/gpucall.out
exit 3
