#!/bin/bash
# GPU box experiment: config-3 kernel time of the default library with the
# port hash dense (<= 32 words) and sparse, alternating, then the stage-ablated
# variants (vpp_amd/variants/lib_abl*.so, tools/build_ablate.sh).
# usage: tools/gpu_exp.sh <tag> [variant libs...]
set -e -o pipefail
TAG=${1:-exp}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for r in 1 2; do
  for d in 1 0; do
    echo "== dense=$d round $r"
    CONTIVCLS_PHASH_DENSE=$d timeout -k 10 200 python tools/ablate.py 3 2>&1 | grep -E "info|kernel median" | sed -e 's/^info.*list_mode.: \([0-9]*\).*/list_mode \1/'
  done
done 2>&1 | tee $OUT/dense.log
if [ $# -gt 0 ]; then
  CONTIVCLS_PHASH_DENSE=0 timeout -k 10 600 python tools/ablate.py 3 vpp_amd/libcontivcls.so "$@" 2>&1 | grep -E "==|kernel median" | tee $OUT/ablate.log
fi
