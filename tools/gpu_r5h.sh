#!/bin/bash
# Round 5: legacy row spans -- legacy parity, then C2 / C3 A/B against libshs_base.so (the commit before),
# interleaved three times (bench --strong '' so only the legacy loop runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_batch.py tests/test_overflow_async.py tests/test_shipped_frames.py tests/test_exp_switches.py > gpurun_out/r5h_tests.log 2>&1 || { tail -40 gpurun_out/r5h_tests.log; exit 1; }
tail -2 gpurun_out/r5h_tests.log
for rep in 1 2 3; do
  for c in c2 c3; do
    for v in base default; do
      L=; [ $v = base ] && L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_base.so
      SHS_GPU_LIB=$L timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 200 --warmup 20 \
        > gpurun_out/r5h_${v}_$c.log 2>&1 || { tail -20 gpurun_out/r5h_${v}_$c.log; exit 1; }
      python - gpurun_out/r5h_${v}_$c.log $v $c <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'))
PY
    done
  done
done
