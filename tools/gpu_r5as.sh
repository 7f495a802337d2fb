#!/bin/bash
# Round 5: upper bound of the legacy pair test's two correctly rounded divisions (libshs_fdiv.so: a
# hardware reciprocal instead, wrong results, timing only), C3 and C2, interleaved twice.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for c in c3 c2; do
    for v in gpu fdiv; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5as_${c}_$v.log 2>&1 || { tail -20 gpurun_out/r5as_${c}_$v.log; exit 1; }
      python3 - gpurun_out/r5as_${c}_$v.log $c $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
