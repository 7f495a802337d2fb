#!/bin/bash
# GPU-box experiment: C2 kernel times under debug flags (outputs are wrong by design for flags != 0).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/flags.log
for f in ${FLAGS:-0x0 0x100 0x200 0x1000 0x400 0x4000 0x4300}; do
  timeout -k 10 120 python bench.py --no-pmc --no-cpu --steps 300 --warmup 30 --debug-flags $f $BENCH_ARGS > gpurun_out/flag_$f.log 2>&1 || { tail -5 gpurun_out/flag_$f.log; exit 1; }
  python -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/flag_$f.log') if l.startswith('{')][-1]
print('$f', d['value'], d['ms_per_step'], d['kernels_ms'])" | tee -a gpurun_out/flags.log
done
