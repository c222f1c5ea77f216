#!/bin/bash
# Host sanitizers (ASan + UBSan) over the rule compiler and the CPU oracle.
# CPU only (runs in the build container).  usage: tools/asan/run.sh
set -e -o pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT=${TMPDIR:-/tmp}/contivcls_asan
mkdir -p $OUT
python3 $HERE/dump_acls.py $OUT/acls.txt
/opt/rocm/lib/llvm/bin/clang -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
    -fno-sanitize-recover=undefined -c -o $OUT/oracle.o $ROOT/oracle/aclengine_ref.c
# host code sanitized; the device code of kernels.hip is compiled without it
CXX=/opt/rocm/lib/llvm/bin/clang++
SAN="-O1 -g -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
OBJS=$OUT/oracle.o
for src in tools/asan/asan_main.cpp vpp_amd/csrc/compile.cpp vpp_amd/csrc/engine.cpp vpp_amd/csrc/kernels.hip; do
    o=$OUT/$(basename $src).o
    $CXX -x hip --offload-arch=gfx950 -std=c++17 $SAN -fno-gpu-sanitize -I$ROOT/include -c -o $o $ROOT/$src &
    PIDS="$PIDS $!"
    OBJS="$OBJS $o"
done
for p in $PIDS; do wait $p; done
$CXX --hip-link --offload-arch=gfx950 $SAN -fno-gpu-sanitize -o $OUT/asan_main $OBJS -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,/opt/rocm/lib
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    $OUT/asan_main $OUT/acls.txt > $OUT/run.log
grep -c 'compile v4 0 v16 0' $OUT/run.log
tail -1 $OUT/run.log
