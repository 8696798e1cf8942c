#!/bin/bash
# build_variant.sh NAME [extra hipcc flags...] -> variants/NAME.so (for tools/ab.py A/B runs)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p variants
C=advancedgraphicsraytracer_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -shared -Wno-unused-function \
  -I $C "$@" -o variants/$name.so -x hip $C/rt_host.cpp $C/rt_device.hip $C/rt_kern_core.hip $C/rt_kern_ext.hip $C/rt_multi.cpp $C/rt_sbvh.cpp -lz -ldl
echo variants/$name.so
