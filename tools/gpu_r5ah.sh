#!/bin/bash
# Round 5: k_lib_setup at a 6-wave bound (libshs_lsw6.so: 80 VGPRs, 7 spilled, 6 workgroups per CU
# instead of 5) against the default: C4 / C5 A/B three times, then the 8-way C4 / C5 split.
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_lsw6.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_fullsize.py > gpurun_out/r5ah_tests.log 2>&1 || { tail -30 gpurun_out/r5ah_tests.log; exit 1; }
tail -1 gpurun_out/r5ah_tests.log
VARIANTS="default lsw6 default lsw6 default lsw6" CONFIGS="c4 c5" bash tools/exp_variants.sh || exit 1
for c in c4 c5; do
  for v in default lsw6; do
    if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
    SHS_GPU_LIB=$L SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 60 8 3 > gpurun_out/r5ah_split_${c}_$v.log 2>&1 || exit 1
    echo "== $c $v"; grep "$c N" gpurun_out/r5ah_split_${c}_$v.log
  done
done
