#!/bin/bash
# Re-submit a gpurun call while the pool answers "no box / transient" (exit 3: nothing ran, nothing
# charged). Any other exit code -- including a failing or faulting GPU step -- is returned as is.
# usage: tools/gpurun_retry.sh <timeout-s> '<command>'
T=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] pool busy/transient (attempt $i); sleeping 60 s"
  sleep 60
done
exit 3
