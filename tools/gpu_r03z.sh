#!/bin/bash
# Round 3: packet-load issue order in classify4_cls (src, dst, dport, proto
# as the stream kernel, CLS_LOAD_ORDER=1) with and without the evaluation,
# against the default and unclamped builds; one process, then the floors.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03z}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
V=vpp_amd/variants
timeout -k 10 500 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so $V/lib_nc.so $V/lib_ordnc.so $V/lib_abl63nc.so $V/lib_abl63ord.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --settle-ms 100 --cpu-sample 0 2>&1 >/dev/null | grep "stream floor"
