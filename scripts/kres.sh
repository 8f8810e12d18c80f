#!/bin/bash
# Register / LDS / scratch use of the kernels of one source file: scripts/kres.sh <file.hip> [name-filter]
cd "$(dirname "$0")/../siddhi_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -x hip -c "$1" -o /tmp/kres.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys, re
for l in sys.stdin:
    m = re.search(r'Name: (\S+)', l)
    if m: print(); print(m.group(1)[:60], end=' ')
    for k in ['VGPRs', 'ScratchSize \[bytes/lane\]', 'Occupancy \[waves/SIMD\]', 'LDS Size \[bytes/block\]']:
        m = re.search(k + r': (\d+)', l)
        if m: print(k.split(' ')[0] + '=' + m.group(1), end=' ')
print()" | grep -E "${2:-.}"
