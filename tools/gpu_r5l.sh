#!/bin/bash
# Round 5: eager normal loads in k_lib_setup (libshs_enrm.so) against the default build -- library
# parity with the variant, C4 / C5 bench A/B, and the 8-way C4 split A/B.
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_enrm.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_spatial_order.py tests/test_textures.py > gpurun_out/r5l_tests.log 2>&1 || { tail -30 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
VARIANTS="default enrm default enrm" CONFIGS="c4 c5" bash tools/exp_variants.sh || exit 1
for v in default enrm default enrm; do
  if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
  SHS_GPU_LIB=$L SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c4 60 8 3 > gpurun_out/r5l_split_$v.log 2>&1 || exit 1
  echo "== $v"; grep "c4 N" gpurun_out/r5l_split_$v.log
done
