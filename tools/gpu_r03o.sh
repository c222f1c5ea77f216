#!/bin/bash
# Round 3: connection batches with the bitmap form of linear IPv4 ACLs --
# the connection GPU tests, then tools/conn_bench.py under rocprofv3 (12 and
# 64 local ACLs, bitmap on / off); then the classify stream-shape A/B
# (tools/gpu_r03n.sh).  usage: tools/gpu_r03o.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03o}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 12 64; do
  for B in 1 0; do
    CONTIVCLS_CONN_BITMAP=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_${L}_$B -o run --output-format csv -- python3 tools/conn_bench.py --locals $L > $OUT/conn${L}_bm$B.json 2> $OUT/conn${L}_bm$B.err
    echo "locals $L bitmap $B"; python tools/kstats.py $OUT/conn_prof_${L}_$B/run_kernel_stats.csv | grep -E "connect|classify4"
    python -c "import json;d=json.load(open('$OUT/conn${L}_bm$B.json'));print(d['hbm_resident'], d['hbm_resident_counted'])"
  done
done
bash tools/gpu_r03n.sh ${TAG}_n
