#!/bin/bash
# Kernel resource usage (VGPR/SGPR/LDS/spills) of mbots_kernels.hip for extra hipcc flags.
#   bash scripts/kres.sh [-DFOO ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d)
(cd $d && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --save-temps "$@" \
    -c $ROOT/madrona-bots_amd/csrc/mbots_kernels.hip -o k.o 2>/dev/null)
python3 - "$d"/mbots_kernels-hip-amdgcn-amd-amdhsa-gfx950.s <<'PY'
import re, sys
s = open(sys.argv[1]).read()
meta = s[s.index('amdhsa.kernels:'):]
for blk in meta.split('\n  - ')[1:]:
    m = re.search(r'\.name:\s+(\S+)', blk)
    if not m:
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\S+)', blk) or [None, '-'])[1]
    print(f"{m.group(1)[8:40]:32s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} "
          f"lds {g('group_segment_fixed_size'):>6} spill {g('vgpr_spill_count')}/{g('sgpr_spill_count')}")
PY
rm -rf $d
