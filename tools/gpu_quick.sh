#!/bin/bash
# GPU box: the GPU test suite (verbose log) and one config-3 bench line.
# usage: tools/gpu_quick.sh <tag> [pytest -k expression]
set -e -o pipefail
TAG=${1:-quick}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
K=${2:-}
echo "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
echo "bench config 3"
timeout -k 10 300 python bench.py > $OUT/bench3.json 2> $OUT/bench3.err
cat $OUT/bench3.json
