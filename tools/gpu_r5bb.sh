#!/bin/bash
# Round 5: the legacy raster at a 5-wave bound (libshs_rw5.so: 96 VGPRs, 15 / 25 spilled) with 5
# workgroups per CU (SHS_RASTER_PER_CU=5) against the default 4 (experiments builds), C2; C3 at its 3
# and at 4 per CU.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag lib per_cu config
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$2.so SHS_RASTER_PER_CU=$3 timeout -k 10 200 python bench.py --config $4 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
    > gpurun_out/r5bb_$1.log 2>&1 || { tail -20 gpurun_out/r5bb_$1.log; exit 1; }
  python3 - gpurun_out/r5bb_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
}
for rep in 1 2; do
  run c2_def_$rep gpu_exp 4 c2 || exit 1
  run c2_rw5_$rep rw5 5 c2 || exit 1
  run c2_rw5x4_$rep rw5 4 c2 || exit 1
  run c3_def_$rep gpu_exp 3 c3 || exit 1
  run c3_rw5x4_$rep rw5 4 c3 || exit 1
done
