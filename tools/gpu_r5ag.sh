#!/bin/bash
# Round 5: k_lib_resolve with each block's coverage flag and winner words loaded a block ahead
# (libshs_rpf.so, -DSHS_RESOLVE_PREFETCH) against the default: library parity with the variant,
# C4 / C5 A/B interleaved three times, then the isolated kernel times.
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_rpf.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_fullsize.py tests/test_shipped_regions.py tests/test_textures.py > gpurun_out/r5ag_tests.log 2>&1 || { tail -30 gpurun_out/r5ag_tests.log; exit 1; }
tail -1 gpurun_out/r5ag_tests.log
VARIANTS="default rpf default rpf default rpf" CONFIGS="c4 c5" bash tools/exp_variants.sh || exit 1
