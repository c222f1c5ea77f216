#!/bin/bash
# Round 3 (session 2): smoke, the whole -m gpu suite, driver-style config-3
# benches, the rocprofv3 kernel summary of the same command, config 5, the
# connection batches and the gen-policy lists.  usage: tools/gpu_r03i.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03i}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
# test failures (rc 1) do not stop the measurements; a crash, abort or time limit does
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
grep -E "FAILED|ERROR" $OUT/pytest.log | head -30 || true
tail -2 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_c3_1.json 2> $OUT/bench_c3_1.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_2.json 2> $OUT/bench_c3_2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_prof.json 2> $OUT/bench_c3_prof.err
python tools/kstats.py $OUT/prof_c3/run_kernel_stats.csv
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
python tools/bsum.py $OUT/bench_*.json
echo "connection batches"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof -o run --output-format csv -- python3 tools/conn_bench.py --locals 12 > $OUT/conn12.json 2> $OUT/conn12.err
python tools/kstats.py $OUT/conn_prof/run_kernel_stats.csv
echo "gen-policy lists"
timeout -k 10 400 python tools/genpolicy_bench.py --blocks 20 200 1000 > $OUT/genpolicy.jsonl 2> $OUT/genpolicy.err
python tools/jl.py $OUT/genpolicy.jsonl workload rules list_mode kernel_ms Gpps_kernel Gpps_wall
