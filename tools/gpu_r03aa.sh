#!/bin/bash
# Round 3: the 16-byte stream shapes of tools/stream16_glds.hip against the
# engine's stream16 floor and classify16_cls, same box.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 60 tools/stream16_glds.bin rand
CONTIVCLS_DEBUG_FLOOR=1 timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-sample 0 2> /tmp/c5.err | python tools/bsum.py /dev/stdin
grep "stream floor" /tmp/c5.err
