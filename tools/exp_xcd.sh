#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# k_lib_raster tile order experiment: bench C4 / C5 per supertile edge (SHS_LIB_XCD_ST).
set -o pipefail
mkdir -p gpurun_out
for c in ${CONFIGS:-c4 c5}; do
  for st in ${STS:-0 1 2 4}; do
    SHS_LIB_XCD_ST=$st timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --steps 100 --warmup 10 \
      > gpurun_out/xcd_${c}_$st.log 2>&1 || { tail -20 gpurun_out/xcd_${c}_$st.log; exit 1; }
    python - gpurun_out/xcd_${c}_$st.log $c $st <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'st', sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
