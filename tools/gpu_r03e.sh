#!/bin/bash
# Round 3: config-3 bench after the mode-6 default-cell fix: mode 6 vs row
# entries vs round-2 form, then the changed GPU tests.  usage: tools/gpu_r03e.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03e}
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
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_trie_wide.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
