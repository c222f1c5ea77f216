#!/bin/bash
# Round 3: defaults back to binary sublists / row entries; config 3 and 5
# benches, gen-policy both forms, connection kernel, then the whole -m gpu
# suite.  usage: tools/gpu_r03h.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03h}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_$i.json 2> $OUT/bench_c3_$i.err
done
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
python tools/bsum.py $OUT/bench_*.json
echo "connection batches"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof -o run --output-format csv -- python3 tools/conn_bench.py --locals 12 > $OUT/conn12.json 2> $OUT/conn12.err
python tools/kstats.py $OUT/conn_prof/run_kernel_stats.csv
echo "gen-policy lists"
timeout -k 10 600 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy.jsonl 2> $OUT/genpolicy.err
CONTIVCLS_SUB4=1 timeout -k 10 600 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy_sub4.jsonl 2> $OUT/genpolicy_sub4.err
python tools/jl.py $OUT/genpolicy.jsonl workload rules list_mode kernel_ms Gpps_kernel Gpps_wall
python tools/jl.py $OUT/genpolicy_sub4.jsonl workload rules list_mode kernel_ms Gpps_kernel Gpps_wall
echo "pytest -m gpu"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
