#!/bin/bash
# Round 5: what the C2 busy tiles spend (experiments build; wrong images): the clear strips skipped
# (DBG_SKIP_CLEAR 0x1000) alone, with the shading skipped (DBG_SKIP_SHADE 0x200), with the pair tests
# skipped (DBG_SKIP_PAIRS 0x4000), and both.  128 frames per step.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for rep in 1 2; do
  for fl in 0x1000 0x1200 0x5000 0x5200 0x200 0x4000; do
    timeout -k 10 200 python bench.py --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5u_$fl.log 2>&1 || { tail -20 gpurun_out/r5u_$fl.log; exit 1; }
    python3 - gpurun_out/r5u_$fl.log $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('flags', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
