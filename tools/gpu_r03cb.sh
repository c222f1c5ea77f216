#!/bin/bash
# Round 3: renderer commit latency on a 1000-pod node (GPU engine).
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/gpurun_out/r03cb
cd $ROOT
timeout -k 10 600 python tools/commit_bench.py --engine gpu > gpurun_out/r03cb/commit_bench.json 2> gpurun_out/r03cb/commit_bench.err
python -c "
import json; d=json.load(open('gpurun_out/r03cb/commit_bench.json'))
for k in ('rules','pods','nochange'): print(k, d[k]['median'])
print('full', d['full_render'])"
