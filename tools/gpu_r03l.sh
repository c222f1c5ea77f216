#!/bin/bash
# Round 3: stage ablation of classify4_cls on config 3 in one process (the
# default build against counting off, sublist probes off, source lookup off,
# port lookup off, all lookups off), then the SQ counter passes of the default
# build.  usage: tools/gpu_r03l.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03l}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
V=vpp_amd/variants
timeout -k 10 500 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so $V/lib_abl1.so $V/lib_abl2.so $V/lib_abl4.so $V/lib_abl8.so $V/lib_abl15.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
timeout -k 10 700 bash tools/sq_profile.sh $TAG
