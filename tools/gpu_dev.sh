#!/bin/bash
# GPU box development check: the whole -m gpu suite, an in-process A/B of
# kernel builds on config 3 (tools/ab_inproc.py), and one bench line.
# usage: tools/gpu_dev.sh <tag> [variant libs for the A/B...]
set -e -o pipefail
TAG=${1:-dev}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
echo "pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
if [ $# -gt 0 ]; then
  echo "A/B"
  timeout -k 10 400 python tools/ab_inproc.py --rounds 8 "$@" vpp_amd/libcontivcls.so > $OUT/ab.log 2>&1
  grep median $OUT/ab.log
fi
echo "bench config 3"
timeout -k 10 300 python bench.py > $OUT/bench3.json 2> $OUT/bench3.err
python -c "import json;d=json.load(open('$OUT/bench3.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms_avg'],r['stream_floor_ms'],r['frac'])"
