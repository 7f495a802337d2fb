#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for sl in ${SLICES:-1 2 4 8}; do
  SHS_EXP_GHOST_SLICES=$sl timeout -k 10 120 python bench.py --no-pmc --no-cpu --steps 100 --warmup 10 $BENCH_ARGS > gpurun_out/sl_$sl.log 2>&1 || { tail -5 gpurun_out/sl_$sl.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/sl_$sl.log') if l.startswith('{')][-1]
print('$sl', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
