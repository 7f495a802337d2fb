#!/bin/bash
# Round 5: k_lib_blocks with 16 lanes per setup block (working tree) against one thread per block
# (libshs_base.so = HEAD): the region-sharded parity tests, then the 8-way split C4 / C5 rank frames.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_regions.py tests/test_shipped_regions.py tests/test_region_balance.py tests/test_shadow_footprint.py \
  > gpurun_out/r5cc_tests.log 2>&1 || { tail -30 gpurun_out/r5cc_tests.log; exit 1; }
tail -3 gpurun_out/r5cc_tests.log
for rep in 1 2; do
  for lib in base gpu; do
    for cfg in c4 c5; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$lib.so SPLIT_REGIONS=1 timeout -k 10 200 \
        python tools/exp_pipeline.py $cfg 60 8 1 > gpurun_out/r5cc_${cfg}_${lib}_$rep.log 2>&1 \
        || { tail -20 gpurun_out/r5cc_${cfg}_${lib}_$rep.log; exit 1; }
      echo "== $cfg $lib $rep"; tail -4 gpurun_out/r5cc_${cfg}_${lib}_$rep.log
    done
  done
done
