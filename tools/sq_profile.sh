#!/bin/bash
# SQ/LDS counter passes of the classify kernel (run on the GPU box).
# usage: tools/sq_profile.sh <tag> [bench.py args]; SQ_CMD="python3 ..." profiles
# another command (e.g. tools/genpolicy_bench.py) instead of bench.py.
set -e -o pipefail
TAG=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B=${SQ_CMD:-"python3 $ROOT/bench.py --steps 2 --warmup 1 --settle-ms 0 --cpu-sample 0 $@"}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT -d $OUT/a -o run --output-format csv -- $B > $OUT/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/b -o run --output-format csv -- $B > $OUT/b.log 2>&1
python3 - "$OUT" "$ROOT" <<'PY'
import csv, collections, sys, glob, os
out = sys.argv[1]
sys.path.insert(0, sys.argv[2])
from vpp_amd._abi import source_hash
KERNELS = os.environ.get("SQ_KERNELS", "classify4_cls,classify16_cls").split(",")
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in KERNELS):
            agg[(r["Kernel_Name"].split("namespace)::")[-1].split("(")[0][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
with open(out + "/summary.txt", "w") as fo:
    fo.write("# kernel sources (vpp_amd/csrc) hash %s\n" % source_hash())
    for k in sorted(agg):
        v = agg[k]
        fo.write("%-60s %-24s %14.0f  (n=%d)\n" % (k[0], k[1], sum(v) / len(v), len(v)))
print(open(out + "/summary.txt").read())
PY
