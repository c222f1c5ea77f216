#!/bin/bash
# GPU box: PMC HBM traffic of the classify kernels (configs 3 and 5) and the
# renderer commit latency at 1000 pods.  usage: tools/gpu_meas.sh <tag>
set -e -o pipefail
TAG=${1:-meas}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
bash tools/gpu_pmc.sh ${TAG}_pmc3 3 > $OUT/pmc3.log 2>&1
bash tools/gpu_pmc.sh ${TAG}_pmc5 5 > $OUT/pmc5.log 2>&1
grep -h ratio $OUT/pmc3.log $OUT/pmc5.log
timeout -k 10 400 python tools/commit_bench.py --pods 1000 --engine gpu > $OUT/commit.json 2> $OUT/commit.err
cat $OUT/commit.json
