#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# Timing A/B of environment switches on one config: ENVS="A=0 A=1" CONFIG=c5 bash tools/exp_env.sh
set -o pipefail
mkdir -p gpurun_out
for e in ${ENVS:-X=0}; do
  env $e timeout -k 10 200 python bench.py --config ${CONFIG:-c5} --no-pmc --no-cpu --no-single --no-pcie --steps 100 --warmup 10 \
    > gpurun_out/env_$e.log 2>&1 || { tail -20 gpurun_out/env_$e.log; exit 1; }
  python - gpurun_out/env_$e.log "$e" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
done
