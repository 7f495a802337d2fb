#!/bin/bash
# k_lib_setup timing experiments (GPU box): the C4 bench's kernel times with parts of the setup skipped
# (SHS_LIB_EXP bits: 1 no LibShade stores, 2 no busy marks / bin appends, 4 no LibRec stores).
set -o pipefail
mkdir -p gpurun_out
for x in 0 1 2 4 7; do
  SHS_LIB_EXP=$x timeout -k 10 200 python bench.py --config c4 --no-pmc --no-cpu --steps 20 --warmup 5 \
    > gpurun_out/exp_lib_$x.log 2>&1 || { tail -5 gpurun_out/exp_lib_$x.log; exit 1; }
  echo "exp=$x $(grep '^{' gpurun_out/exp_lib_$x.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms"])')"
done
