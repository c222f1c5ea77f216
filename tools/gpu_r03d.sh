#!/bin/bash
# Round 3: why is src mode 6 (inline cells) slower?  SQ counters and timing of
# mode 6 against row entries (CONTIVCLS_INLINE=0).  usage: tools/gpu_r03d.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03d}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_m6.json 2> $OUT/bench_m6.err
CONTIVCLS_SUB4=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_m6_bin.json 2> $OUT/bench_m6_bin.err
CONTIVCLS_INLINE=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_rows.json 2> $OUT/bench_rows.err
python tools/bsum.py $OUT/bench_*.json
bash tools/sq_profile.sh ${TAG}_m6
CONTIVCLS_INLINE=0 bash tools/sq_profile.sh ${TAG}_rows
