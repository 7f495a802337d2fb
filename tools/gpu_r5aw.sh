#!/bin/bash
# Round 5: debug-flag code compiled only into the experiments build (working tree) against HEAD
# (libshs_base.so): legacy parity, C3 / C2 A/B interleaved three times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch.py tests/test_shipped_frames.py > gpurun_out/r5aw_tests.log 2>&1 || { tail -30 gpurun_out/r5aw_tests.log; exit 1; }
tail -1 gpurun_out/r5aw_tests.log
for rep in 1 2 3; do
  for c in c3 c2; do
    for v in base gpu; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5aw_${c}_$v.log 2>&1 || { tail -20 gpurun_out/r5aw_${c}_$v.log; exit 1; }
      python3 - gpurun_out/r5aw_${c}_$v.log $c $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
