#!/bin/bash
# GPU-box check: parity tests, one bench line, rocprofv3 kernel stats.
# usage: tools/gpu_check.sh <tag>
set -e -o pipefail
TAG=${1:-run}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $ROOT/bench.py --cpu-sample 0 > $OUT/stats.log 2>&1
find $OUT -name "*kernel_stats.csv" -exec cat {} \;
