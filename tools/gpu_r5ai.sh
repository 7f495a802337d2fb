#!/bin/bash
# Round 5: sliver walks over conservative line spans (working tree) against HEAD (libshs_base.so):
# the whole -m gpu suite, then C2 / C3 A/B interleaved three times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5ai_tests.log 2>&1 || { tail -30 gpurun_out/r5ai_tests.log; exit 1; }
tail -1 gpurun_out/r5ai_tests.log
for rep in 1 2 3; do
  for c in c3 c2; do
    for v in base gpu; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --config $c --no-pmc --no-cpu --no-pcie --strong '' --steps 100 --warmup 10 \
        > gpurun_out/r5ai_${c}_$v.log 2>&1 || { tail -20 gpurun_out/r5ai_${c}_$v.log; exit 1; }
      python3 - gpurun_out/r5ai_${c}_$v.log $c $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'), 'single', d.get('single_frame', {}).get('ms_per_frame'))
PY
    done
  done
done
