#!/bin/bash
# Round 3: config-3 bench A/B after the mode-6 fix (mode 6 / row entries /
# round-2 form), the connection kernel with LDS-staged tables, then the
# changed GPU tests.  usage: tools/gpu_r03g.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03g}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_m6_$i.json 2> $OUT/bench_m6_$i.err
  CONTIVCLS_INLINE=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_rows_$i.json 2> $OUT/bench_rows_$i.err
  CONTIVCLS_INLINE=0 CONTIVCLS_SUB4=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_r2_$i.json 2> $OUT/bench_r2_$i.err
done
python tools/bsum.py $OUT/bench_*.json
echo "connection batches"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof -o run --output-format csv -- python3 tools/conn_bench.py --locals 12 > $OUT/conn12.json 2> $OUT/conn12.err
CONTIVCLS_CONN_NO_LDS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_gmeta -o run --output-format csv -- python3 tools/conn_bench.py --locals 12 > $OUT/conn12_gmeta.json 2> $OUT/conn12_gmeta.err
python tools/kstats.py $OUT/conn_prof/run_kernel_stats.csv $OUT/conn_prof_gmeta/run_kernel_stats.csv
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_trie_wide.py tests/test_gpu_connect_scale.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
