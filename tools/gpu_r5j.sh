#!/bin/bash
# Round 5: the whole -m gpu suite, then C2 with 64 / 128 / 256 frames per step (interleaved twice).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  > gpurun_out/r5j_tests.log 2>&1 || { tail -40 gpurun_out/r5j_tests.log; exit 1; }
tail -2 gpurun_out/r5j_tests.log
for rep in 1 2; do
  for F in 64 128 256; do
    timeout -k 10 200 python bench.py --frames-per-step $F --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5j_c2_$F.log 2>&1 || { tail -20 gpurun_out/r5j_c2_$F.log; exit 1; }
    python3 - gpurun_out/r5j_c2_$F.log $F <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('F', sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'), 'frac', d['roofline']['frac'], d['roofline']['step_frac'])
PY
  done
done
