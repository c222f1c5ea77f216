#!/bin/bash
# Round-3 first GPU check: the changed GPU tests, then bench as the driver
# runs it (--steps 20 --warmup 5) and with 25 warm-up steps, twice each.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/r03a
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_acl_config.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_w5_$i.json 2> $OUT/bench_w5_$i.err
  timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_w25_$i.json 2> $OUT/bench_w25_$i.err
done
python tools/bsum.py $OUT/bench_w*.json
