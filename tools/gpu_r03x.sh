#!/bin/bash
# Round 3: the stream floor shapes with a 125 KB dynamic LDS allocation (as
# the config-3 classify launch) against none.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT
export TMPDIR=/tmp
for L in 0 128320 0 128320; do
  echo "dynamic LDS $L"
  CONTIVCLS_FLOOR_LDS=$L CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --settle-ms 100 --cpu-sample 0 2>&1 >/dev/null | grep "stream floor"
done
