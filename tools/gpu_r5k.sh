#!/bin/bash
# Round 5: C2 k_raster with the busy tiles' stores dropped (DBG_SKIP_TILE_STORES, experiments build;
# wrong images) against the same build without the flag, interleaved twice.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for rep in 1 2; do
  for fl in 0 0x8000 0x400; do
    timeout -k 10 200 python bench.py --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5k_$fl.log 2>&1 || { tail -20 gpurun_out/r5k_$fl.log; exit 1; }
    python3 - gpurun_out/r5k_$fl.log $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('flags', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
