#!/bin/bash
# Round 5: scan mode as a compile-time raster parameter (working tree) against HEAD (libshs_base.so),
# and scan-mode frames on row spans (libshs_sspan.so, -DSHS_SCAN_SPANS): legacy parity of both,
# then C2 (and C3 for the default) A/B three times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch.py tests/test_shipped_frames.py > gpurun_out/r5av_tests.log 2>&1 || { tail -30 gpurun_out/r5av_tests.log; exit 1; }
tail -1 gpurun_out/r5av_tests.log
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_sspan.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch.py tests/test_shipped_frames.py > gpurun_out/r5av_tests_sspan.log 2>&1 || { tail -30 gpurun_out/r5av_tests_sspan.log; exit 1; }
tail -1 gpurun_out/r5av_tests_sspan.log
for rep in 1 2 3; do
  for v in base gpu sspan; do
    SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so timeout -k 10 200 python bench.py --config c2 --no-pmc --no-cpu --no-pcie --strong '' --steps 100 --warmup 10 \
      > gpurun_out/r5av_c2_$v.log 2>&1 || { tail -20 gpurun_out/r5av_c2_$v.log; exit 1; }
    python3 - gpurun_out/r5av_c2_$v.log c2 $v <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], 'ms/step', d['ms_per_step'], 'kernels', d.get('kernels_ms'), 'single', d.get('single_frame', {}).get('ms_per_frame'))
PY
  done
done
