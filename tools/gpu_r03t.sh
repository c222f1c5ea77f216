#!/bin/bash
# Round 3: connection kernel with every call's descriptor and slot word
# loaded up front (CONN_PREFETCH=1) against the default build: per-call wall
# times and kernel stats on the 12- and 64-local conn_bench setups.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03t}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for L in 12 64; do
  for V in default cpf; do
    if [ $V = default ]; then LIB=$ROOT/vpp_amd/libcontivcls.so; else LIB=$ROOT/vpp_amd/variants/lib_$V.so; fi
    CONTIVCLS_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p_${L}_$V -o run --output-format csv -- python3 tools/conn_bench.py --locals $L --cpu-sample 200 > $OUT/c${L}_$V.json 2> $OUT/c${L}_$V.err
    echo "locals $L $V"; python tools/kstats.py $OUT/p_${L}_$V/run_kernel_stats.csv | grep -E "connect_kernel<false, true"
    python -c "import json;d=json.load(open('$OUT/c${L}_$V.json'));print(d['hbm_resident'], d['hbm_resident_counted'])"
  done
done
