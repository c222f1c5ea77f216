#!/bin/bash
# Round 3: the classify loop's stream shape -- protocol loads non-temporal
# (CLS_NT_PROTO=1), alone and with the one-step prefetch (CLS_PREFETCH=1) or
# the ordered prefetch (CLS_PREFETCH=3) -- against the default build on
# config 3, one process; the per-shape stream floors of the same box.
# usage: tools/gpu_r03n.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03n}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
V=vpp_amd/variants
timeout -k 10 500 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so $V/lib_nt.so $V/lib_pf1nt.so $V/lib_pf3nt.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_c3.json 2> $OUT/b_c3.err
grep "stream floor" $OUT/b_c3.err || true
python tools/bsum.py $OUT/b_*.json
