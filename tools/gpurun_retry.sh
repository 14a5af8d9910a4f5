#!/bin/bash
# usage: gpurun_retry.sh <log> <timeout> <cmd...>: retries only while gpurun reports no free slot (exit 3)
log=$1; shift; to=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "done rc=$rc" >> $log; exit $rc; fi
  echo "no slot (try $i)" >> $log.tries
  sleep 120
done
echo "done rc=3 (gave up)" >> $log
