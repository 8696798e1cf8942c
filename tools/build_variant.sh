#!/bin/bash
# build_variant.sh NAME [DEVICE_SRC] [extra hipcc flags...] -> variants/NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=advancedgraphicsraytracer_amd/csrc/rt_device.hip
if [ $# -gt 0 ] && [ -f "$1" ]; then src=$1; shift; fi
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-function \
  -I advancedgraphicsraytracer_amd/csrc "$@" -o variants/$name.so advancedgraphicsraytracer_amd/csrc/rt_host.cpp "$src" -lz
echo variants/$name.so
