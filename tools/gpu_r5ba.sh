#!/bin/bash
# Round 5: C2 with the unbounded slivers listed for k_ghost (SHS_GHOST_LIST=1, experiments build) against
# the inline walks in the setup waves (default), now that the walks are span-cut; interleaved three times.
set -o pipefail
mkdir -p gpurun_out
export SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so
for rep in 1 2 3; do
  for g in 0 1; do
    SHS_GHOST_LIST=$g timeout -k 10 200 python bench.py --config c2 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5ba_$g.log 2>&1 || { tail -20 gpurun_out/r5ba_$g.log; exit 1; }
    python3 - gpurun_out/r5ba_$g.log $g <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('ghost_list', sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
