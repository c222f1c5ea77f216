#!/bin/bash
# Round-3 GPU measurements then tests.  usage: tools/gpu_r03c.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/${1:-r03c}
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
echo "bench config 3"
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_w5_$i.json 2> $OUT/bench_w5_$i.err
  CONTIVCLS_SUB4=0 CONTIVCLS_INLINE=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_r2_w5_$i.json 2> $OUT/bench_r2_w5_$i.err
  CONTIVCLS_INLINE=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_sub4_w5_$i.json 2> $OUT/bench_sub4_w5_$i.err
done
timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_w25.json 2> $OUT/bench_w25.err
python tools/bsum.py $OUT/bench_w*.json $OUT/bench_r2*.json $OUT/bench_sub4*.json
echo "connection batches"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof -o run --output-format csv -- python3 tools/conn_bench.py --locals 12 > $OUT/conn12.json 2> $OUT/conn12.err
CONTIVCLS_CONN_SORTED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_perlane -o run --output-format csv -- python3 tools/conn_bench.py --locals 12 > $OUT/conn12_perlane.json 2> $OUT/conn12_perlane.err
cat $OUT/conn12.json $OUT/conn12_perlane.json
echo "gen-policy lists"
timeout -k 10 600 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy.jsonl 2> $OUT/genpolicy.err
python tools/jl.py $OUT/genpolicy.jsonl workload rules list_mode lds_slots slots kernel_ms Gpps_kernel Gpps_wall
echo "LDS-DMA stream experiment"
timeout -k 10 120 ./tools/stream_glds.bin > $OUT/stream_glds.txt 2>&1
cat $OUT/stream_glds.txt
timeout -k 10 180 ./tools/stream16_glds.bin > $OUT/stream16_glds.txt 2>&1
cat $OUT/stream16_glds.txt
echo "pytest (changed GPU tests)"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_connect_scale.py tests/test_gpu_trie_wide.py tests/test_gpu_sessions.py tests/test_gpu_acl_config.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
