#!/bin/bash
# Round 5: the legacy setup on the raster's own stream (SHS_LEGACY_ONE_STREAM=1, experiments build)
# against the two-stream default, C2 and C3, interleaved twice.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for rep in 1 2; do
  for c in c2 c3; do
    for o in 0 1; do
      SHS_LEGACY_ONE_STREAM=$o timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5af_${c}_$o.log 2>&1 || { tail -20 gpurun_out/r5af_${c}_$o.log; exit 1; }
      python3 - gpurun_out/r5af_${c}_$o.log $c $o <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'one_stream', sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
