#!/bin/bash
# GPU box: where a config-2 step goes (16 Mi packets, the kernel ~40 us):
# driver-flag bench lines (default, one workgroup per CU) and the kernel trace
# of the same command with the gaps between launches (tools/gaps.py).
# usage: tools/gpu_cfg2.sh <tag>
set -e -o pipefail
TAG=${1:-cfg2}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
B="--config 2 --steps 20 --warmup 5 --cpu-sample 0"
timeout -k 10 200 python bench.py $B > $OUT/b2.json 2> $OUT/b2.err
python3 tools/jl.py $OUT/b2.json value ms_per_step step_ms_median host_submit_ms_per_step roofline.kernel_ms_median roofline.stream_floor_ms
CONTIVCLS_WG_PER_CU=1 timeout -k 10 200 python bench.py $B > $OUT/b2_wg1.json 2> $OUT/b2_wg1.err
python3 tools/jl.py $OUT/b2_wg1.json value ms_per_step step_ms_median host_submit_ms_per_step roofline.kernel_ms_median
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ROOT/bench.py $B > $OUT/kt.log 2>&1
python3 $ROOT/tools/gaps.py $(find $OUT/kt -name "run_kernel_trace.csv") --last 120
