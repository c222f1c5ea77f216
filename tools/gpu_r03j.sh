#!/bin/bash
# Round 3: in-process A/B of the ordered-prefetch build (CLS_PREFETCH=3) and
# the build without the 4-ary sublist branch against the default library on
# config 3; bench.py under several step / warm-up / settle settings; the
# counter-tier GPU tests.  usage: tools/gpu_r03j.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03j}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for a in memset rand; do
  timeout -k 10 60 tools/stream_glds.bin $a > $OUT/stream_glds_$a.txt 2>&1
  timeout -k 10 60 tools/stream16_glds.bin $a > $OUT/stream16_glds_$a.txt 2>&1
done
head -30 $OUT/stream_glds_*.txt $OUT/stream16_glds_*.txt
timeout -k 10 400 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so vpp_amd/variants/lib_nos4.so vpp_amd/variants/lib_pf3.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_s20w5.json 2> $OUT/b.err
timeout -k 10 200 python bench.py --steps 50 --warmup 25 --cpu-sample 0 > $OUT/b_s50w25.json 2>> $OUT/b.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --settle-ms 0 --cpu-sample 0 > $OUT/b_s20w5_nosettle.json 2>> $OUT/b.err
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --cpu-sample 0 > $OUT/b_s200w5.json 2>> $OUT/b.err
CONTIVCLS_LIB=$ROOT/vpp_amd/variants/lib_pf3.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_pf3_s20w5.json 2>> $OUT/b.err
python tools/bsum.py $OUT/b_*.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_counters.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
