#!/bin/bash
# gpuq.sh NAME TIMEOUT SCRIPT: one gpurun call of SCRIPT, re-submitted only while the pool
# has no free box (transient / exit 3: nothing ran, nothing charged); output -> gpurun_out/NAME.out
set -u
name=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > gpurun_out/$name.out 2>&1; rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" gpurun_out/$name.out; then sleep 150; continue; fi
  exit $rc
done
