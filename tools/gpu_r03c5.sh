#!/bin/bash
# Round 3, final sources: rocprofv3 kernel summary of the config-5 bench and
# the SQ counters of classify16_cls.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/r03c5
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run --output-format csv -- python3 bench.py --config 5 --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c5_prof.json 2> $OUT/bench.err
python tools/kstats.py $OUT/prof_c5/run_kernel_stats.csv
timeout -k 10 300 bash tools/sq_profile.sh r03c5 --config 5
