#!/bin/bash
# Round 5: C3 after the legacy row spans -- per-workgroup timeline of one frame and the PMC passes of a
# 16-frame step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/timeline.py c3 > gpurun_out/r5i_tl_c3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5i_tl_c3.log | tail -30
timeout -k 10 500 bash tools/pmc_kernels.sh r5i_c3 --config c3 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_r5i_c3.json'))
for k,v in d.items(): print(k[:40], {c: v[c] for c in ('fetch_bytes_x2','write_bytes','valu_active_per_wave_cycle','wait_any_frac') if c in v})
"
