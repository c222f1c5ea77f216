#!/bin/bash
# GPU box: connection-batch bench (12 and 64 local ACLs) with rocprofv3 kernel
# stats of the 12-local run.  usage: tools/gpu_conn_prof.sh <tag>
set -e -o pipefail
TAG=${1:-conn}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python tools/conn_bench.py --locals 64 > $OUT/conn64.json 2> $OUT/conn64.err
python3 tools/jl.py $OUT/conn64.json value hbm_resident hbm_resident_counted
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p12 -o run --output-format csv -- python3 $ROOT/tools/conn_bench.py --locals 12 > $OUT/conn12.json 2> $OUT/conn12.err
python3 $ROOT/tools/jl.py $OUT/conn12.json value hbm_resident hbm_resident_counted
python3 $ROOT/tools/kstats.py $OUT/p12/run_kernel_stats.csv
