#!/bin/bash
# Round 3: connection kernel ablation (no evaluation / descriptor reads only
# / no bitmap evaluation) on the 12- and 64-local conn_bench, kernel stats.
# usage: tools/gpu_r03q.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03q}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for L in 12 64; do
  for V in default cabl1 cabl2 cabl4; do
    if [ $V = default ]; then LIB=$ROOT/vpp_amd/libcontivcls.so; else LIB=$ROOT/vpp_amd/variants/lib_$V.so; fi
    CONTIVCLS_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p_${L}_$V -o run --output-format csv -- python3 tools/conn_bench.py --locals $L --count 0 --cpu-sample 200 > $OUT/c${L}_$V.json 2> $OUT/c${L}_$V.err || true
    echo "locals $L $V"; python tools/kstats.py $OUT/p_${L}_$V/run_kernel_stats.csv | grep -E "connect_kernel<false, true"
  done
done
