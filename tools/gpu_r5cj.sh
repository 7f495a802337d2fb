#!/bin/bash
# Round 5: C2 in bin mode (--raster-mode 2: per-bin-tile candidate lists, row spans) against scan mode
# (the default for scenes up to 4,096 triangles), two A/B pairs.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag mode
  timeout -k 10 200 python bench.py --config c2 --raster-mode $2 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 200 --warmup 10 \
    > gpurun_out/r5cj_$1.log 2>&1 || { tail -20 gpurun_out/r5cj_$1.log; exit 1; }
  python3 - gpurun_out/r5cj_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'value', d['value'], 'kernels', d.get('kernels_ms'))
PY
}
for rep in 1 2; do
  run scan_$rep 0 || exit 1
  run bins_$rep 2 || exit 1
done
