#!/bin/bash
# Round 3 final checks, part 2: config 2 and config 4 (N = 1) bench lines,
# the gen-policy lists, connection batches (12 / 64 local ACLs) with kernel
# stats.  usage: tools/gpu_r03v.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03v}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c2.json 2> $OUT/bench.err
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --cpu-sample 0 > $OUT/bench_c4.json 2>> $OUT/bench.err
python tools/bsum.py $OUT/bench_*.json
for L in 12 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_$L -o run --output-format csv -- python3 tools/conn_bench.py --locals $L > $OUT/conn$L.json 2> $OUT/conn$L.err
  echo "locals $L"; python tools/kstats.py $OUT/conn_prof_$L/run_kernel_stats.csv | grep -E "conn|classify4"
  python -c "import json;d=json.load(open('$OUT/conn$L.json'));print(d['hbm_resident'], d['hbm_resident_counted'], d['value'], d['cpu_baseline'])"
done
timeout -k 10 500 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy.jsonl 2> $OUT/genpolicy.err
python tools/jl.py $OUT/genpolicy.jsonl workload rules list_mode kernel_ms Gpps_kernel Gpps_wall
