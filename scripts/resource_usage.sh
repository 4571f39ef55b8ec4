#!/bin/bash
# VGPR / AGPR / spill / occupancy of the life kernels in one variant TU
# (hipcc -Rpass-analysis=kernel-resource-usage).  Usage:
#   scripts/resource_usage.sh [variant=bits_w1_dpp] [name-filter=.]
set -euo pipefail
cd "$(dirname "$0")/.."
V=${1:-bits_w1_dpp}
F=${2:-.}
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Icsrc/include -Icsrc \
  -mllvm -amdgpu-sched-strategy=${GOL_SCHED_STRATEGY:-max-ilp} ${EXTRA_FLAGS:-} \
  -Rpass-analysis=kernel-resource-usage -c "csrc/kernels/life_block_${V}.hip" -o /tmp/ru_$$.o 2> /tmp/ru_$$.txt
python3 - "$F" /tmp/ru_$$.txt <<'EOF'
import re, sys
flt, path = sys.argv[1], sys.argv[2]
for b in re.split(r'remark: .*?Function Name: ', open(path).read())[1:]:
    name = b.split('\n')[0].split(' ')[0]
    if not re.search(flt, name):
        continue
    g = lambda k: (re.search(re.escape(k) + r': (\S+)', b) or [None, '-'])[1]
    lds, occ = g('LDS Size [bytes/block]'), g('Occupancy [waves/SIMD]')
    print(f"{name[14:70]:56s} vgpr {g('VGPRs'):>4} agpr {g('AGPRs'):>4} spill {g('VGPRs Spill'):>4} "
          f"lds {lds:>6} occ {occ}")
EOF
rm -f /tmp/ru_$$.o /tmp/ru_$$.txt
