#!/bin/bash
# Host-side AddressSanitizer run (no GPU: CPU mode only) of the cross-capacity
# checkpoint save / load and mbots_max_population through the C ABI
# (tests/c_host/cap_asan.c), against a libmbots built with -Xarch_host
# -fsanitize=address (the device code is not instrumented).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d)
(cd $ROOT/madrona-bots_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC \
    -ffp-contract=off -fno-slp-vectorize -Xarch_host -fsanitize=address -shared -o $d/libmbots_asan.so \
    mbots_kernels.hip mbots_manager.cpp mbots_cpu.cpp)
/opt/rocm/llvm/bin/clang -g -fsanitize=address -std=c99 -I$ROOT/include $ROOT/tests/c_host/cap_asan.c \
    -L$d -lmbots_asan -Wl,-rpath,$d -o $d/cap_asan
ASAN_OPTIONS=detect_leaks=0 $d/cap_asan
rm -rf $d
