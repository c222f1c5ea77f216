#!/bin/bash
# Round 3: the classify loop without evaluation (abl63) against the same
# without the load clamps (abl63nc), without the prologue / epilogue (abl127),
# and the full kernel without the clamps (nc); one process, then the floors.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03y}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
V=vpp_amd/variants
timeout -k 10 500 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so $V/lib_nc.so $V/lib_abl63.so $V/lib_abl63nc.so $V/lib_abl127.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --settle-ms 100 --cpu-sample 0 2>&1 >/dev/null | grep "stream floor"
