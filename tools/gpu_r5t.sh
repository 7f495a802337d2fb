#!/bin/bash
# Round 5: the deep camera raster's next-pass record prefetch (libshs_pf4.so: -DSHS_LIB_PREFETCH, 4-wave
# bound) against the default build and the 4-wave bound alone (libshs_w4.so): library parity with the
# variant, C4 / C5 bench A/B, and the 8-way split (SPLIT_REGIONS=1).
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_pf4.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_fullsize.py tests/test_shipped_regions.py tests/test_spatial_order.py > gpurun_out/r5t_tests.log 2>&1 || { tail -30 gpurun_out/r5t_tests.log; exit 1; }
tail -1 gpurun_out/r5t_tests.log
VARIANTS="default w4 pf4 default w4 pf4" CONFIGS="c4 c5" bash tools/exp_variants.sh || exit 1
for v in default pf4 w4; do
  if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
  SHS_GPU_LIB=$L SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c4 60 8 3 > gpurun_out/r5t_split_$v.log 2>&1 || exit 1
  echo "== $v"; grep "c4 N" gpurun_out/r5t_split_$v.log
done
