#!/bin/bash
# Build an A/B variant of libmbots.so: build_var.sh NAME KERNELS_FILE [extra hipcc flags]
# (kernels file replaces csrc/mbots_kernels.hip; the manager is the tree's).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; src=$2; shift 2
d=$ROOT/build_var/src_$name
mkdir -p $d
cp "$src" $d/mbots_kernels.hip
cp $ROOT/madrona-bots_amd/csrc/{mbots_manager.cpp,mbots_cpu.cpp,mbots_cpu.hpp,mbots_device.hpp,mbots_kernels.hpp,mbots_ray.hpp} $d/
(cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize "$@" \
    -shared -o $ROOT/build_var/libmbots_$name.so mbots_kernels.hip mbots_manager.cpp mbots_cpu.cpp)
rm -rf $d
