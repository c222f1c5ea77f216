#!/bin/bash
# GPU box: A/B of kernel build variants (vpp_amd/variants/lib_*.so, built
# with make -C vpp_amd/csrc variant V=<name> F=<flags>) against the default
# library: config 3 via tools/ablate.py, config 5 via bench.py.
# usage: tools/gpu_ab.sh <tag> <variant names for config 3> -- <variant names for config 5>
set -e -o pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
V3=(); V5=(); cur=3
for a in "$@"; do
    if [ "$a" = "--" ]; then cur=5; continue; fi
    if [ $cur = 3 ]; then V3+=("$a"); else V5+=("$a"); fi
done
LIBS="vpp_amd/libcontivcls.so"
for v in "${V3[@]}"; do LIBS="$LIBS vpp_amd/variants/lib_$v.so"; done
timeout -k 10 400 python tools/ablate.py 3 $LIBS > $OUT/ab3.log 2>&1
grep -E "==|kernel median" $OUT/ab3.log
if [ ${#V5[@]} -gt 0 ]; then
    timeout -k 10 300 python bench.py --config 5 --steps 10 --cpu-sample 0 > $OUT/b5_default.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/b5_default.json'));print('default', d['roofline']['kernel_ms_avg'], d['roofline']['stream_floor_ms'])"
    for v in "${V5[@]}"; do
        CONTIVCLS_LIB=$ROOT/vpp_amd/variants/lib_$v.so timeout -k 10 300 python bench.py --config 5 --steps 10 --cpu-sample 0 > $OUT/b5_$v.json 2>/dev/null
        python -c "import json;d=json.load(open('$OUT/b5_$v.json'));print('$v', d['roofline']['kernel_ms_avg'])"
    done
fi
