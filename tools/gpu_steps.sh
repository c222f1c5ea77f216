#!/bin/bash
# GPU box: run steps in order, each under its own time limit; stop at the
# first step that faulted, aborted or timed out (exit 124/134/137/139 or a
# signal).  A step that merely fails (e.g. pytest exit 1) is reported and the
# next step still runs.
# usage: tools/gpu_steps.sh <tag> <seconds> '<cmd>' [<seconds> '<cmd>' ...]
# each command's output goes to gpurun_out/<tag>/step<k>.log
TAG=$1
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 2
k=0
while [ $# -ge 2 ]; do
    secs=$1
    cmd=$2
    shift 2
    k=$((k + 1))
    echo "== step $k: $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/step$k.log" 2>&1
    rc=$?
    tail -25 "$OUT/step$k.log"
    echo "== step $k rc=$rc"
    case $rc in
        0|1|2|5) ;;
        *) echo "stopping: step $k ended with $rc"; exit $rc ;;
    esac
done
