#!/bin/bash
# Round-3 GPU check: changed GPU tests, bench as the driver runs it, gen-policy lists.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r03b}
mkdir -p $OUT
cd $ROOT
echo "pytest (changed GPU tests)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_connect_scale.py tests/test_gpu_trie_wide.py tests/test_gpu_sessions.py tests/test_gpu_acl_config.py tests/test_gpu_parity.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_w5_$i.json 2> $OUT/bench_w5_$i.err
  timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_w25_$i.json 2> $OUT/bench_w25_$i.err
  CONTIVCLS_SUB4=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_bin_w5_$i.json 2> $OUT/bench_bin_w5_$i.err
done
python tools/bsum.py $OUT/bench_w*.json $OUT/bench_bin*.json
echo "gen-policy lists"
timeout -k 10 600 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy.jsonl 2> $OUT/genpolicy.err
python tools/jl.py $OUT/genpolicy.jsonl workload rules list_mode lds_slots slots kernel_ms Gpps_kernel Gpps_wall
echo "connection batches (sorted kernel, then the per-lane kernel)"
timeout -k 10 300 python tools/conn_bench.py --locals 12 > $OUT/conn12.json 2> $OUT/conn12.err
CONTIVCLS_CONN_SORTED=0 timeout -k 10 300 python tools/conn_bench.py --locals 12 > $OUT/conn12_perlane.json 2> $OUT/conn12_perlane.err
cat $OUT/conn12.json $OUT/conn12_perlane.json
