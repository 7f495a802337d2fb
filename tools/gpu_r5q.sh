#!/bin/bash
# Round 5: clear-strip item height 1 / 2 / 4 / 8 raster-tile rows (libshs_st{1,2,4}.so, default 8),
# C2 at 128 frames per step, and the busy tiles alone (DBG_SKIP_CLEAR, experiments build).
set -o pipefail
mkdir -p gpurun_out
run() {   # name lib flags
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$2.so timeout -k 10 200 python bench.py --debug-flags $3 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
    > gpurun_out/r5q_$1.log 2>&1 || { tail -20 gpurun_out/r5q_$1.log; exit 1; }
  python3 - gpurun_out/r5q_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
B=d['roofline']['algorithmic_bytes']; k=d['kernels_ms']['raster']
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'), 'raster TB/s', round(B/k/1e9, 2))
PY
}
for rep in 1 2; do
  for v in gpu st1 st2 st4; do run ${v}_$rep $v 0 || exit 1; done
  run skipclr_$rep gpu_exp 0x1000 || exit 1
done
