#!/bin/bash
# Round 3: depth-specialised kernels without the run-time 4-ary branch;
# A/B of the ordered prefetch (CLS_PREFETCH=3, one and two packet groups per
# lane) on config 3; bench lines for config 3 (default, pf3) and config 5;
# the GPU tests touched by the change.  usage: tools/gpu_r03k.sh <tag>
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03k}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_inproc.py --config 3 --rounds 8 vpp_amd/libcontivcls.so vpp_amd/variants/lib_pf3.so vpp_amd/variants/lib_pf3g2.so > $OUT/ab3.txt 2>&1
cat $OUT/ab3.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_c3.json 2> $OUT/b.err
CONTIVCLS_LIB=$ROOT/vpp_amd/variants/lib_pf3.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_c3_pf3.json 2>> $OUT/b.err
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-sample 0 > $OUT/b_c5.json 2>> $OUT/b.err
python tools/bsum.py $OUT/b_*.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_v16.py tests/test_gpu_trie_wide.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
