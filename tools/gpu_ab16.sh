#!/bin/bash
# GPU box: A/B of the 16-byte kernel's packet order (config 5), parity first.
#   tools/gpu_ab16.sh <tag>   (build vpp_amd/variants/lib_c0.so with
#   make -C vpp_amd/csrc variant V=c0 F=-DCLS_COAL16=0 beforehand)
set -e -o pipefail
TAG=${1:-ab16}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_v16.py tests/test_gpu_traffic.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --config 5 --steps 10 --cpu-sample 0 > $OUT/bench5_new.json 2> $OUT/bench5_new.err
cat $OUT/bench5_new.json
CONTIVCLS_LIB=$ROOT/vpp_amd/variants/lib_c0.so timeout -k 10 300 python bench.py --config 5 --steps 10 --cpu-sample 0 > $OUT/bench5_old.json 2> $OUT/bench5_old.err
cat $OUT/bench5_old.json
bash tools/gpu_pmc.sh ${TAG}_pmc5 5
