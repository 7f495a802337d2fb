#!/bin/bash
# Round 5: the region-sharded camera setup as its own k_lib_setup instance at six waves per SIMD
# (working tree) against five (libshs_r5w.so) and HEAD (libshs_base.so: one instance, five waves):
# the region parity tests, then the 8-way split C4 / C5 at three frames in flight and C4 at N = 1.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_regions.py tests/test_shipped_regions.py tests/test_region_balance.py tests/test_shadow_footprint.py \
  > gpurun_out/r5cd_tests.log 2>&1 || { tail -30 gpurun_out/r5cd_tests.log; exit 1; }
tail -1 gpurun_out/r5cd_tests.log
for rep in 1 2; do
  for lib in base gpu r5w; do
    for cfg in c4 c5; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$lib.so SPLIT_REGIONS=1 timeout -k 10 200 \
        python tools/exp_pipeline.py $cfg 60 8 3 > gpurun_out/r5cd_${cfg}_${lib}_$rep.log 2>&1 \
        || { tail -20 gpurun_out/r5cd_${cfg}_${lib}_$rep.log; exit 1; }
      echo "== $cfg $lib $rep"; grep "per-rank" gpurun_out/r5cd_${cfg}_${lib}_$rep.log
    done
  done
  for lib in base gpu; do
    SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$lib.so SPLIT_REGIONS=1 timeout -k 10 200 \
      python tools/exp_pipeline.py c4 60 1 3 > gpurun_out/r5cd_n1_${lib}_$rep.log 2>&1 \
      || { tail -20 gpurun_out/r5cd_n1_${lib}_$rep.log; exit 1; }
    echo "== n1 $lib $rep"; grep "per-rank" gpurun_out/r5cd_n1_${lib}_$rep.log
  done
done
