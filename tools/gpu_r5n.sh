#!/bin/bash
# Round 5: C2 clear-only (DBG_CLEAR_ONLY) and the real raster at 64 / 128 / 256 frames per step
# (experiments build): the store rate per batch size.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for F in 64 128 256; do
  for fl in 0 0x400; do
    timeout -k 10 200 python bench.py --frames-per-step $F --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5n_${F}_$fl.log 2>&1 || { tail -20 gpurun_out/r5n_${F}_$fl.log; exit 1; }
    python3 - gpurun_out/r5n_${F}_$fl.log $F $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
B=d['roofline']['algorithmic_bytes']; k=d['kernels_ms']['raster']
print('F', sys.argv[2], 'flags', sys.argv[3], 'ms/step', d['ms_per_step'], 'raster ms', k, 'TB/s', round(B/k/1e9, 2))
PY
  done
done
