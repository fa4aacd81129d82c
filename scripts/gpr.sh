#!/bin/bash
# gpurun with retries while no GPU slot is free (exit code 3: nothing ran, nothing charged)
log=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $log; then exit $rc; fi
  sleep 90
done
exit 3
