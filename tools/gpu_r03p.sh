#!/bin/bash
# Round 3: split connection path (conn_eval_kernel + conn_state_kernel) --
# connection GPU tests, then conn_bench under rocprofv3 (12 / 64 locals,
# split on / off).  usage: tools/gpu_r03p.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03p}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py tests/test_gpu_parity.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 12 64; do
  for S in 1 0; do
    CONTIVCLS_CONN_SPLIT=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_${L}_$S -o run --output-format csv -- python3 tools/conn_bench.py --locals $L > $OUT/conn${L}_split$S.json 2> $OUT/conn${L}_split$S.err
    echo "locals $L split $S"; python tools/kstats.py $OUT/conn_prof_${L}_$S/run_kernel_stats.csv | grep -E "conn|classify4"
    python -c "import json;d=json.load(open('$OUT/conn${L}_split$S.json'));print(d['hbm_resident'], d['hbm_resident_counted'])"
  done
done
