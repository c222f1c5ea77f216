#!/bin/bash
# GPU box: PMC HBM traffic (configs 3 and 5) and the SQ/LDS counter passes
# of config 3, each rocprofv3 --pmc pass a run of its own.
# usage: tools/gpu_counters.sh <tag>
set -e -o pipefail
TAG=${1:-ctr}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT
bash tools/gpu_pmc.sh ${TAG}_pmc3 3 > /dev/null 2>&1
bash tools/gpu_pmc.sh ${TAG}_pmc5 5 > /dev/null 2>&1
grep -h "ratio\|source_hash" gpurun_out/${TAG}_pmc3/pmc.json gpurun_out/${TAG}_pmc5/pmc.json
bash tools/sq_profile.sh ${TAG} > /dev/null 2>&1
cat gpurun_out/sq_${TAG}/summary.txt
