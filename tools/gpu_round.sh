#!/bin/bash
# GPU-box round check: parity tests, bench lines for configs 3 and 5, and
# rocprofv3 kernel stats for both.  Every GPU step has its own time limit and
# the script stops at the first failure.
# usage: tools/gpu_round.sh <tag>
set -e -o pipefail
TAG=${1:-run}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
echo "pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
echo "bench config 3"
timeout -k 10 300 python bench.py > $OUT/bench3.json 2> $OUT/bench3.err
cat $OUT/bench3.json
echo "bench config 5"
timeout -k 10 300 python bench.py --config 5 --steps 10 > $OUT/bench5.json 2> $OUT/bench5.err
cat $OUT/bench5.json
export TMPDIR=/tmp
cd /tmp
echo "rocprof config 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats3 -o run --output-format csv -- python3 $ROOT/bench.py --cpu-sample 0 > $OUT/stats3.log 2>&1
echo "rocprof config 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats5 -o run --output-format csv -- python3 $ROOT/bench.py --config 5 --steps 10 --cpu-sample 0 > $OUT/stats5.log 2>&1
find $OUT -name "*kernel_stats.csv" -exec cat {} \;
