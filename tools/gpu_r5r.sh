#!/bin/bash
# Round 5: C2 k_raster with the clear strips skipped (DBG_SKIP_CLEAR, experiments build; wrong images):
# the busy tiles alone, against the full raster, 64 and 128 frames per step.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for F in 128 64; do
  for fl in 0 0x1000 0x400; do
    timeout -k 10 200 python bench.py --frames-per-step $F --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5r_${F}_$fl.log 2>&1 || { tail -20 gpurun_out/r5r_${F}_$fl.log; exit 1; }
    python3 - gpurun_out/r5r_${F}_$fl.log $F $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('F', sys.argv[2], 'flags', sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
