#!/bin/bash
# Round 5: plain framebuffer stores in the legacy raster and clears (libshs_plain.so,
# -DSHS_LEGACY_PLAIN_STORES) against the non-temporal default: C2 / C3 A/B pairs, then the legacy
# parity tests with the plain build.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag lib config
  SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$2.so timeout -k 10 200 python bench.py --config $3 --no-pmc --no-cpu --no-single --no-pcie --strong '' --steps 200 --warmup 10 \
    > gpurun_out/r5ci_$1.log 2>&1 || { tail -20 gpurun_out/r5ci_$1.log; exit 1; }
  python3 - gpurun_out/r5ci_$1.log $1 <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'value', d['value'], 'kernels', d.get('kernels_ms'), 'frac', d['roofline']['frac'])
PY
}
for rep in 1 2 3; do
  run c2_nt_$rep gpu c2 || exit 1
  run c2_plain_$rep plain c2 || exit 1
  run c3_nt_$rep gpu c3 || exit 1
  run c3_plain_$rep plain c3 || exit 1
done
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_plain.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_batch.py tests/test_shipped_frames.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5ci_tests.log 2>&1 || { tail -30 gpurun_out/r5ci_tests.log; exit 1; }
tail -1 gpurun_out/r5ci_tests.log
