#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# Library setup cost split (timing only; SHS_LIB_EXP makes wrong images): no LibShade stores (1),
# no marks / bin appends (2), no LibRec stores (4), at full C4 and as rank 0 of 8.
set -o pipefail
mkdir -p gpurun_out
for f in 0 1 4 5 2; do
  SHS_LIB_EXP=$f timeout -k 10 200 python bench.py --config c4 --no-pmc --no-cpu --no-single --no-pcie --steps 50 --warmup 5 \
    > gpurun_out/expf_$f.log 2>&1 || { tail -5 gpurun_out/expf_$f.log; exit 1; }
  python - gpurun_out/expf_$f.log $f <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('SHS_LIB_EXP', sys.argv[2], 'ms/step', d['ms_per_step'], d.get('kernels_ms'))
PY
done
