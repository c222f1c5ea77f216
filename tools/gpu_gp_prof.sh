#!/bin/bash
# GPU box: per-kernel times (rocprofv3) of the gen-policy bench on one list
# (--blocks B, ingress) for the current library and each variant given.
# usage: tools/gpu_gp_prof.sh <tag> <blocks> [variant libs...]
set -e -o pipefail
TAG=${1:-gpprof}; B=${2:-20}; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for lib in vpp_amd/libcontivcls.so "$@"; do
  i=$((i+1))
  CONTIVCLS_LIB=$ROOT/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python3 $ROOT/tools/genpolicy_bench.py --blocks $B --match ingress --iters 5 > $OUT/p$i.log 2>&1
  echo "== $lib"
  grep workload $OUT/p$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['rules'], d['Gpps_wall'], d['kernel_ms'], d['Gpps_kernel'])"
  find $OUT/p$i -name "*kernel_stats.csv" -exec cat {} \; | grep -E "classify|finish|other|fold|remap" | cut -d, -f1-4 | cut -c1-160
done
