#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# Timing attribution with debug flags (wrong images): CONFIG=c3 FLAGS="0 0x800" bash tools/exp_flags.sh
# (DBG_SKIP_GHOST 0x100, DBG_SKIP_SHADE 0x200, DBG_CLEAR_ONLY 0x400, DBG_SKIP_BIN 0x800, DBG_SKIP_CLEAR 0x1000)
set -o pipefail
mkdir -p gpurun_out
for f in ${FLAGS:-0}; do
  timeout -k 10 200 python bench.py --config ${CONFIG:-c3} --no-pmc --no-cpu --no-single --no-pcie --steps 100 --warmup 10 --debug-flags $f \
    > gpurun_out/flags_$f.log 2>&1 || { tail -5 gpurun_out/flags_$f.log; exit 1; }
  python - gpurun_out/flags_$f.log $f <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('flags', sys.argv[2], 'ms/step', d['ms_per_step'], d.get('kernels_ms'))
PY
done
