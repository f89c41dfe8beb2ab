#!/bin/bash
# Re-request a GPU box when gpurun reports an infrastructure event (status=transient / exit 3:
# nothing ran, nothing charged). Any other outcome — including a failing command — is final.
# usage: tools/gpurun_retry.sh <log> <timeout-seconds> '<command>'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $log; then
    echo "transient (attempt $i), retrying in 60 s" >> $log.retries
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
