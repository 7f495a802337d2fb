#!/bin/bash
# Round 5: clear-strip item height against the clears alone (DBG_CLEAR_ONLY 0x400) and the full raster,
# experiments builds of 1 / 4 / 8 (default) raster-tile rows per item, C2.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in gpu_exp exst4 exst1; do
    for fl in 0x400 0; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --debug-flags $fl --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5an_${v}_$fl.log 2>&1 || { tail -20 gpurun_out/r5an_${v}_$fl.log; exit 1; }
      python3 - gpurun_out/r5an_${v}_$fl.log $v $fl <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'flags', sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
