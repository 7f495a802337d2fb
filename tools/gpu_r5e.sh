#!/bin/bash
# Round 5: candidate-range split tiles (SHS_OPT_LIB_PART) -- parity, then the 8-way C4 / C5 split on one
# GPU per part size (0 = off).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_spatial_order.py tests/test_regions.py \
  > gpurun_out/r5e_tests.log 2>&1 || { tail -40 gpurun_out/r5e_tests.log; exit 1; }
tail -2 gpurun_out/r5e_tests.log
for part in 0 1024 512 256; do
  for c in c4 c5; do
    SPLIT_PART=$part SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 60 1,8 3 > gpurun_out/r5e_split_${c}_$part.log 2>&1 || exit 1
    echo "== $c part $part"; grep "$c N" gpurun_out/r5e_split_${c}_$part.log
  done
done
