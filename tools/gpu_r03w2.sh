#!/bin/bash
# Round 3, final sources: config 2 and config 4 (N = 1) lines, the gen-policy
# lists, and two more driver-style config-3 lines.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03fin5}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_a.json 2> $OUT/bench.err
timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c2.json 2>> $OUT/bench.err
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --cpu-sample 0 > $OUT/bench_c4.json 2>> $OUT/bench.err
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_b.json 2>> $OUT/bench.err
python tools/bsum.py $OUT/bench_*.json
timeout -k 10 500 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy.jsonl 2> $OUT/genpolicy.err
python tools/jl.py $OUT/genpolicy.jsonl workload rules list_mode kernel_ms Gpps_kernel Gpps_wall
