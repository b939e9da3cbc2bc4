#!/bin/bash
# usage: gpu_retry.sh OUTFILE 'command' — retries only while gpurun says no box/slot (exit 3)
OUT=$1; shift
for i in $(seq 1 20); do
  timeout 2400 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > $OUT 2>&1
  rc=$?
  echo "exit $rc (attempt $i)" >> $OUT
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
