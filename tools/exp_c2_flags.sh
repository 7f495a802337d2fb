#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# C2 k_raster split (timing only; debug flags make wrong images): default, busy tiles cleared instead
# of rastered (DBG_CLEAR_ONLY 0x400), no clear strips (DBG_SKIP_CLEAR 0x1000).
set -o pipefail
mkdir -p gpurun_out
for f in 0 0x400 0x1000; do
  timeout -k 10 200 python bench.py --config c2 --no-pmc --no-cpu --no-single --no-pcie --steps 200 --warmup 20 --debug-flags $f \
    > gpurun_out/c2f_$f.log 2>&1 || { tail -5 gpurun_out/c2f_$f.log; exit 1; }
  python - gpurun_out/c2f_$f.log $f <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('flags', sys.argv[2], 'ms/step', d['ms_per_step'], d.get('kernels_ms'))
PY
done
