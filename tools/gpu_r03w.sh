#!/bin/bash
# Round 3: where the last 6 % of classify4_cls goes -- the default build
# against every lookup, staging and flush off (abl31) and the whole per-packet
# evaluation off (abl63: the stream kernel's mix in the classify loop), one
# process; then the per-shape stream floors of the same box.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03w}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
V=vpp_amd/variants
timeout -k 10 500 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so $V/lib_abl31.so $V/lib_abl63.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_c3.json 2> $OUT/b_c3.err
grep "stream floor" $OUT/b_c3.err || true
python tools/bsum.py $OUT/b_*.json
