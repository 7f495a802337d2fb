#!/bin/bash
# Legacy change A/B: legacy parity tests with the default build, then C3 (and C2) timing of the
# default build against shs_gpu/libshs_base.so (the previous commit) and ENV_OFF (the new path's
# switch turned off), interleaved twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py \
  tests/test_batch.py tests/test_overflow_async.py tests/test_shard.py tests/test_abi.py} > gpurun_out/lab_tests.log 2>&1 || { tail -40 gpurun_out/lab_tests.log; exit 1; }
tail -2 gpurun_out/lab_tests.log
for rep in 1 2; do
  for c in ${CONFIGS:-c3}; do
    for v in base default off; do
      L=; E=X=0
      [ $v = base ] && L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_base.so
      [ $v = off ] && E=${ENV_OFF:-X=0}
      env $E SHS_GPU_LIB=$L timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --steps 100 --warmup 10 \
        > gpurun_out/lab_${v}_$c.log 2>&1 || { tail -20 gpurun_out/lab_${v}_$c.log; exit 1; }
      python - gpurun_out/lab_${v}_$c.log $v $c <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
