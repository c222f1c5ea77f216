#!/bin/bash
# Round 3 final checks on the final sources (as gpu_r03fin.sh without the A/B, plus the connection benches):
# smoke; the whole -m gpu suite; config-3 bench lines
# (driver flags) and the rocprofv3 kernel summary of the same command; PMC
# traffic passes for configs 3 and 5 (installed under profiles/ so the
# following lines carry roofline.traffic); final config 3 / 5 lines; SQ
# counters of config 3.  usage: tools/gpu_r03fin.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03fin}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp


timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
rc=0
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || rc=$?
grep -E "FAILED|ERROR" $OUT/pytest.log | head -30 || true
tail -2 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_prof.json 2> $OUT/bench.err
python tools/kstats.py $OUT/prof_c3/run_kernel_stats.csv
timeout -k 10 300 bash tools/gpu_pmc.sh ${TAG}_pmc3 3
timeout -k 10 300 bash tools/gpu_pmc.sh ${TAG}_pmc5 5
cp $ROOT/gpurun_out/${TAG}_pmc3/pmc.json $ROOT/profiles/pmc_r03_config3.json
cp $ROOT/gpurun_out/${TAG}_pmc5/pmc.json $ROOT/profiles/pmc_r03_config5.json
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c3_final.json 2>> $OUT/bench.err
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/bench_c3_final2.json 2>> $OUT/bench.err
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 > $OUT/bench_c5_final.json 2>> $OUT/bench.err
python tools/bsum.py $OUT/bench_*.json
timeout -k 10 300 bash tools/sq_profile.sh ${TAG}
for L in 12 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/conn_prof_$L -o run --output-format csv -- python3 tools/conn_bench.py --locals $L > $OUT/conn$L.json 2> $OUT/conn$L.err
  echo "locals $L"; python tools/kstats.py $OUT/conn_prof_$L/run_kernel_stats.csv | grep -E "conn|classify4"
  python -c "import json;d=json.load(open('$OUT/conn$L.json'));print(d['hbm_resident'], d['hbm_resident_counted'])"
done
