#!/bin/bash
# Run on the GPU box: rocprofv3 kernel stats + separate PMC passes for the bench.
# usage: tools/profile.sh <tag> [bench args...]
set -e -o pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="$@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $ROOT/bench.py $ARGS --cpu-sample 0 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d $OUT/sq -o run --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/sq2.log 2>&1
find $OUT -name "*.csv" | head -50
