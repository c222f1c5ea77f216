#!/bin/bash
# Host side (this container): run one gpurun call, and if no box or slot was
# free (exit 3: nothing ran, nothing charged) try again after a pause, a few
# times.  Any other exit -- including a failing or faulting GPU step -- ends
# it: a GPU step is never repeated.
# usage: tools/gpurun_retry.sh <out file> <gpurun timeout s> '<command>'
OUT=$1
T=$2
CMD=$3
for attempt in 1 2 3 4 5 6; do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$OUT" 2>&1
    rc=$?
    echo "attempt $attempt rc=$rc" >> "$OUT"
    [ $rc -ne 3 ] && exit $rc
    sleep 100
done
exit 3
