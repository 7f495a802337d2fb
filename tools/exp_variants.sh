#!/bin/bash
# Compile-time variant timing: bench the given configs with each in-tree library build
# (shs_gpu/libshs_<v>.so; "default" = libshs_gpu.so).  usage: VARIANTS="default sw6" CONFIGS="c4" bash tools/exp_variants.sh
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  for c in ${CONFIGS:-c4}; do
    if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
    SHS_GPU_LIB=$L timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --steps 100 --warmup 10 \
      > gpurun_out/var_${v}_$c.log 2>&1 || { tail -20 gpurun_out/var_${v}_$c.log; exit 1; }
    python - gpurun_out/var_${v}_$c.log $v $c <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
  done
done
