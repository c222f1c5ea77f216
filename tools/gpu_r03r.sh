#!/bin/bash
# Round 3: connection kernel with the bitmap header in the descriptor and
# lock-step interval searches -- connection GPU tests, conn_bench under
# rocprofv3 (12 / 64 local ACLs).  usage: tools/gpu_r03r.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03r}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_connect_scale.py tests/test_gpu_policy_chain.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 12 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_$L -o run --output-format csv -- python3 tools/conn_bench.py --locals $L > $OUT/conn$L.json 2> $OUT/conn$L.err
  echo "locals $L"; python tools/kstats.py $OUT/conn_prof_$L/run_kernel_stats.csv | grep -E "conn|classify4"
  python -c "import json;d=json.load(open('$OUT/conn$L.json'));print(d['hbm_resident'], d['hbm_resident_counted'])"
done
