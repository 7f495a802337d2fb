#!/bin/bash
# C3 legacy k_setup attribution (GPU box): bench kernel times with the ghost waves / bin appends skipped
# (debug flags; timing only, wrong images).
set -o pipefail
mkdir -p gpurun_out
for f in 0 0x100 0x800 0x900; do
  timeout -k 10 200 python bench.py --config c3 --no-pmc --no-cpu --no-single --no-pcie --steps 20 --warmup 5 --debug-flags $f \
    > gpurun_out/exp_c3_$f.log 2>&1 || { tail -5 gpurun_out/exp_c3_$f.log; exit 1; }
  echo "flags=$f $(grep '^{' gpurun_out/exp_c3_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms"], d["ms_per_step"], d["batch_stats"]["ghost_fragments"])')"
done
