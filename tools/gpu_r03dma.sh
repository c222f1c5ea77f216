#!/bin/bash
# Round 3: classify4_cls with the src / dst stream staged through LDS-DMA
# (CLS_DMA=1) against the default build, config 3, one process.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03dma}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so vpp_amd/variants/lib_dma.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
