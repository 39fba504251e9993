#!/bin/bash
# Register use of every kernel in csrc/hpccg_kernels.hip (compiler remarks):
# "VGPRs SGPRs waves/SIMD scratch  kernel". Usage: tools/vgprs.sh [filter-regex]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/hpccg-sycl_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -D__HIP_PLATFORM_AMD__ \
    --offload-arch=gfx950 -c csrc/hpccg_kernels.hip -o /tmp/vgprs_k.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk '/Function Name:/ {name=$(NF-1)}
         /remark:     VGPRs:/ {v=$(NF-1)}
         /remark:     SGPRs:/ {s=$(NF-1)}
         /ScratchSize/ {sc=$(NF-1)}
         /Occupancy/ {print v, s, $(NF-1), sc, name}' |
    c++filt | sed -e 's/hpccg::(anonymous namespace):://' -e 's/(hpccg::CgArgs, bool)//' |
    grep -E "${1:-.}"
