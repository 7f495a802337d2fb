#!/bin/bash
# Round 5: C3 raster workgroups per CU (SHS_RASTER_PER_CU, experiments build; default 3 in bin mode)
# after the spill-free raster and the leaner bin-mode setup.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for rep in 1 2; do
  for r in 3 4 2; do
    SHS_RASTER_PER_CU=$r timeout -k 10 200 python bench.py --config c3 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5ab_$r.log 2>&1 || { tail -20 gpurun_out/r5ab_$r.log; exit 1; }
    python3 - gpurun_out/r5ab_$r.log $r <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('c3 per-cu', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
