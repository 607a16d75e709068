#!/bin/bash
# A/B of prebuilt libraries: ab_libs.sh ROUNDS lib1.so lib2.so ... [-- kbench args]
# (each round runs every library once, interleaved, so drift hits all alike)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in $(seq 1 $rounds); do
  for lib in "${libs[@]}"; do
    MBOTS_LIB=$lib timeout -k 10 120 python scripts/run_variant.py scripts/kbench.py --no-kernel-timing "$@" || exit 1
  done
done
