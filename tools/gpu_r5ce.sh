#!/bin/bash
# Round 5: where C3's k_raster goes -- the experiments build with one debug switch at a time (wrong
# images, timing only): none, DBG_SKIP_PAIRS 0x4000, DBG_SKIP_SHADE 0x200, DBG_SKIP_TILE_STORES 0x8000,
# DBG_SKIP_CLEAR 0x1000, DBG_SKIP_GHOST 0x100.
set -o pipefail
mkdir -p gpurun_out
for fl in 0 0x4000 0x200 0x8000 0x1000 0x100 0; do
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so timeout -k 10 200 python bench.py --config c3 --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
    > gpurun_out/r5ce_$fl.log 2>&1 || { tail -20 gpurun_out/r5ce_$fl.log; exit 1; }
  python3 - gpurun_out/r5ce_$fl.log $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('flags', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
done
