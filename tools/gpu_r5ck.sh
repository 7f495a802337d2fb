#!/bin/bash
# Round 5: camera passes up to 16,384 triangles load their varyings beside the positions
# (k_lib_setup<false, false, true>; working tree) against HEAD (libshs_base.so): the library parity
# tests, then C5 at N = 1 and the 8-way C5 split at three frames in flight, interleaved A/B pairs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_lib_parity.py tests/test_regions.py tests/test_shadow_footprint.py tests/test_fullsize.py tests/test_light_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5ck_tests.log 2>&1 || { tail -30 gpurun_out/r5ck_tests.log; exit 1; }
tail -1 gpurun_out/r5ck_tests.log
for rep in 1 2; do
  for lib in base gpu; do
    SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$lib.so SPLIT_REGIONS=1 timeout -k 10 200 \
      python tools/exp_pipeline.py c5 60 1,8 3 > gpurun_out/r5ck_${lib}_$rep.log 2>&1 || { tail -20 gpurun_out/r5ck_${lib}_$rep.log; exit 1; }
    echo "== $lib $rep"; grep "per-rank" gpurun_out/r5ck_${lib}_$rep.log
  done
done
