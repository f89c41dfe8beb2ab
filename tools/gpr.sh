#!/bin/bash
# Local helper: one gpurun call, re-submitted only while the pool reports no free box / a transient lease failure
# (exit 3 or status=transient: the command did not run and nothing was charged). Any other outcome is final.
#   bash tools/gpr.sh LOG --timeout S -- 'cmd'
log=$1
shift
rc=0
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    sleep 45
    continue
  fi
  break
done
echo "GPR_EXIT $rc" >> "$log"
