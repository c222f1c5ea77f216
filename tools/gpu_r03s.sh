#!/bin/bash
# Round 3: wall time of each device connection batch (64 and 12 local ACLs).
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/conn_calls.py --locals 64
timeout -k 10 200 python tools/conn_calls.py --locals 12
