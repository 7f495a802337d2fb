#!/bin/bash
# Round 5: the raster's last 2 / 4 / 8 x G items busy tiles only (libshs_tail{2,4,8}.so) against the
# proportional interleave (default), C2 and C3, interleaved twice; parity of tail4 first.
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_tail4.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch.py tests/test_shipped_frames.py > gpurun_out/r5ar_tests.log 2>&1 || { tail -30 gpurun_out/r5ar_tests.log; exit 1; }
tail -1 gpurun_out/r5ar_tests.log
for rep in 1 2; do
  for c in c3 c2; do
    for v in gpu tail2 tail4 tail8; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5ar_${c}_$v.log 2>&1 || { tail -20 gpurun_out/r5ar_${c}_$v.log; exit 1; }
      python3 - gpurun_out/r5ar_${c}_$v.log $c $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
