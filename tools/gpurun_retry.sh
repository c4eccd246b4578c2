#!/bin/bash
# Retry a gpurun call ONLY when the harness reports an infrastructure
# transient (exit 3 / status=transient: no box, nothing ran, nothing charged).
# Usage: tools/gpurun_retry.sh LOGFILE TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "[retry] attempt $attempt transient (rc=$rc); sleeping" >> "$log.retries"
    sleep 45
    continue
  fi
  exit $rc
done
exit $rc
