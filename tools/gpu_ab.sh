#!/bin/bash
# GPU box: one-process A/B of classify kernel builds (tools/ab_inproc.py)
# against the default library, config 3 and/or 5.  Variants are built on the
# CPU first: make -C vpp_amd/csrc variant V=<name> F=<flags>, or a copy of an
# older build under vpp_amd/variants/.
# usage: tools/gpu_ab.sh <tag> <config> <variant .so> ...
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python tools/ab_inproc.py --config $CFG --rounds 8 vpp_amd/libcontivcls.so "$@" > $OUT/ab$CFG.log 2>&1
grep -E "median|mismatch|differ" $OUT/ab$CFG.log
