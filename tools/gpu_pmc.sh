#!/bin/bash
# GPU box: HBM traffic of classify4_cls (FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes).  usage: tools/gpu_pmc.sh <tag> [config]
set -e -o pipefail
TAG=${1:-pmc}
CFG=${2:-3}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="$ROOT/bench.py --config $CFG --steps 2 --warmup 1 --settle-ms 0 --cpu-sample 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B > $OUT/write.log 2>&1
N=$(grep '^{"metric"' $OUT/fetch.log | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['config']['packets_per_gpu'])")
python3 $ROOT/tools/pmc_traffic.py pmc $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") $CFG $N $OUT/pmc.json
