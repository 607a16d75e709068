#!/bin/bash
# Build libmbots.so of a git ref (committed csrc) as an A/B variant:
#   build_ref.sh NAME REF [extra hipcc flags]   -> build_var/libmbots_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; ref=$2; shift 2
d=$ROOT/build_var/src_$name
rm -rf $d; mkdir -p $d/x/y/csrc $d/x/include
for f in mbots_kernels.hip mbots_manager.cpp mbots_cpu.cpp mbots_cpu.hpp mbots_device.hpp mbots_kernels.hpp mbots_ray.hpp; do
  git -C $ROOT show $ref:madrona-bots_amd/csrc/$f > $d/x/y/csrc/$f
done
git -C $ROOT show $ref:include/mbots.h > $d/x/include/mbots.h
(cd $d/x/y/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize "$@" \
    -shared -o $ROOT/build_var/libmbots_$name.so mbots_kernels.hip mbots_manager.cpp mbots_cpu.cpp)
rm -rf $d
