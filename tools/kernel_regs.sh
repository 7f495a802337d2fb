#!/bin/bash
# VGPR / SGPR / scratch / LDS / occupancy per kernel of one HIP source, as the compiler reports them
# (-Rpass-analysis=kernel-resource-usage), built with the library's flags plus EXTRA.
# usage: tools/kernel_regs.sh [csrc/file.hip] [kernel name filter] [EXTRA flags]
SRC=${1:-csrc/shs_lib.hip}
FLT=${2:-}
cd "$(dirname "$0")/../leisure-software-renderer_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  $3 --cuda-device-only -c -o /dev/null -Rpass-analysis=kernel-resource-usage "$SRC" 2>&1 | python3 -c "
import sys, re
flt = sys.argv[1]
cur = None
row = {}
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m: cur = m.group(1); continue
    m = re.search(r'remark:\s+(VGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|VGPRs Spill): (\d+)', line)
    if m and cur and flt in cur:
        row.setdefault(cur, []).append(f'{m.group(1).split()[0]}={m.group(2)}')
for k, v in row.items():
    print(f'{k[:70]:70s} ' + ' '.join(v))
" "$FLT"
