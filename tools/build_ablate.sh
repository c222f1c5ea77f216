#!/bin/bash
# Build stage-ablated kernel variants into vpp_amd/variants/ (CPU, hipcc).
set -e
cd "$(dirname "$0")/../vpp_amd/csrc"
for a in ${@:-0 1 2 4 7 15}; do make -s variant V=abl$a F="-DCLS_ABLATE=$a"; done
ls ../variants
