#!/bin/bash
# Round 5: clear strips with each item's busy flags loaded before its stores (working tree) against
# HEAD (libshs_base.so), strip items of 4 / 16 raster-tile rows, and clear-only (DBG_CLEAR_ONLY,
# experiments builds) before/after.  C2, 128 frames per step.
set -o pipefail
mkdir -p gpurun_out
run() {   # name lib flags
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$2.so timeout -k 10 200 python bench.py --debug-flags $3 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
    > gpurun_out/r5o_$1.log 2>&1 || { tail -20 gpurun_out/r5o_$1.log; exit 1; }
  python3 - gpurun_out/r5o_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
B=d['roofline']['algorithmic_bytes']; k=d['kernels_ms']['raster']
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'), 'raster TB/s', round(B/k/1e9, 2))
PY
}
for rep in 1 2; do
  run base_$rep base 0 || exit 1
  run cur_$rep gpu 0 || exit 1
  run st4_$rep st4 0 || exit 1
  run st16_$rep st16 0 || exit 1
  run baseclr_$rep baseexp 0x400 || exit 1
  run curclr_$rep gpu_exp 0x400 || exit 1
done
