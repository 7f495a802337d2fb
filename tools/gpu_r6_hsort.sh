#!/bin/bash
# Round 6: depth-sorted bin lists (k_lib_hsort).  Library parity (new sorted-list tests, full-size C4 / C5,
# region shards), then the hot tiles of rank 3 / 6 of 8 and the C4 / C5 splits against HEAD~1 (libshs_base.so).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_sorted_lists.py \
  tests/test_fullsize.py tests/test_shipped_regions.py tests/test_regions.py tests/test_spatial_order.py tests/test_lib_parity.py \
  > gpurun_out/r6h_tests.log 2>&1 || { tail -40 gpurun_out/r6h_tests.log; exit 1; }
tail -1 gpurun_out/r6h_tests.log
timeout -k 10 240 python -u tools/exp_hot_tiles.py 8 3,6 6 > gpurun_out/r6h_hot8.log 2>&1 || { tail -30 gpurun_out/r6h_hot8.log; exit 1; }
grep -E "rep|wg " gpurun_out/r6h_hot8.log | head -30
for rep in 1 2; do
  for lib in base gpu; do
    for c in c4 c5; do
      SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$lib.so SPLIT_REGIONS=1 timeout -k 10 240 \
        python -u tools/exp_pipeline.py $c 60 1,8 3 > gpurun_out/r6h_${c}_${lib}_$rep.log 2>&1 || { tail -30 gpurun_out/r6h_${c}_${lib}_$rep.log; exit 1; }
      echo "== $c $lib $rep"; grep "per-rank" gpurun_out/r6h_${c}_${lib}_$rep.log
    done
  done
done
