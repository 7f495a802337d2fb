#!/bin/bash
# C2 k_raster time split (GPU box, timing only): normal, busy tiles cleared only (0x400), strips skipped
# (0x1000), both.
set -o pipefail
mkdir -p gpurun_out
for f in ${FLAGS:-0 0x400 0x1000 0x1400}; do
  timeout -k 10 200 python bench.py --config c2 --no-pmc --no-cpu --no-single --no-pcie --steps 50 --warmup 10 --debug-flags $f \
    > gpurun_out/exp_c2_$f.log 2>&1 || { tail -5 gpurun_out/exp_c2_$f.log; exit 1; }
  echo "flags=$f $(grep '^{' gpurun_out/exp_c2_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms"], d["ms_per_step"], d["roofline"]["frac"])')"
done
