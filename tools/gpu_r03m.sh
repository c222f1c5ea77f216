#!/bin/bash
# Round 3: config-3 bench with the per-shape stream floors; the classify
# kernel against itself with every lookup off (abl15) and with the LDS image
# staging and counter flush off too (abl31), in one process; config 5 bench.
# usage: tools/gpu_r03m.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03m}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/b_c3.json 2> $OUT/b_c3.err
grep "stream floor" $OUT/b_c3.err || true
V=vpp_amd/variants
timeout -k 10 500 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so $V/lib_abl15.so $V/lib_abl31.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_c5.json 2> $OUT/b_c5.err
grep "stream floor" $OUT/b_c5.err || true
python tools/bsum.py $OUT/b_*.json
