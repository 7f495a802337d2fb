#!/bin/bash
# Round 5: legacy raster loop, per-pixel (SHS_OPT_RASTER_LOOP 0) vs pair tasks (1, default), C2 and C3.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for c in c2 c3; do
    for l in 1 0; do
      timeout -k 10 200 python bench.py --config $c --raster-loop $l --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5v_${c}_$l.log 2>&1 || { tail -20 gpurun_out/r5v_${c}_$l.log; exit 1; }
      python3 - gpurun_out/r5v_${c}_$l.log $c $l <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'loop', sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
