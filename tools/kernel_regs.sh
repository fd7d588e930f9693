#!/bin/bash
# Register / spill summary per kernel of one source: tools/kernel_regs.sh <file.hip> [-Dmacro ...]
f=$1; shift
out=/tmp/kregs_$$.s
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S "$@" -o $out mysticeti_amd/csrc/$f 2>/dev/null || exit 1
python3 - $out <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)\.vgpr_spill_count:\s+(\d+)', s, re.S):
    pass
for blk in s.split('  - .agpr_count')[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', blk) or [None, '?'])[1]
    print(f"{name[:70]:70s} vgpr={g('vgpr_count')} spill={g('vgpr_spill_count')} priv={g('private_segment_fixed_size')} lds={g('group_segment_fixed_size')}")
PY
rm -f $out
