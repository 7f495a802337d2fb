#!/bin/bash
# Timing sweep over debug flags (phase attribution); prints config, flags, ms/frame, kernel ms (HIP events)
# usage: CFGS="c2 c1" FLAGS="0x0 0x100" bash tools/sweep.sh
for cfg in ${CFGS:-c2}; do
for f in ${FLAGS:-0x0 0x100 0x200 0x400 0x1000}; do
  timeout -k 10 120 python bench.py --config $cfg --no-cpu --no-pmc --steps 100 --warmup 10 --debug-flags $f > gpurun_out/sweep_${cfg}_$f.json 2>&1 || { echo "fail $cfg $f"; tail -3 gpurun_out/sweep_${cfg}_$f.json; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_${cfg}_$f.json')); print('$cfg', '$f', d['ms_per_step'], d['kernels_ms'])"
done; done
