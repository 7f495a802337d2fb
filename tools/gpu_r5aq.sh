#!/bin/bash
# Round 5: Forward+ light direction by one reciprocal (libshs_lrcp.so, -DSHS_LIGHT_RCP) instead of
# three divisions: full-size C4 / C5 parity with the variant (HDR within 1e-5), then C4 A/B.
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_lrcp.so timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_fullsize.py tests/test_lib_parity.py tests/test_light_parity.py > gpurun_out/r5aq_tests.log 2>&1 || { tail -30 gpurun_out/r5aq_tests.log; exit 1; }
grep -E "not bit-identical|passed|failed" gpurun_out/r5aq_tests.log | tail -5
VARIANTS="default lrcp default lrcp default lrcp" CONFIGS="c4" bash tools/exp_variants.sh || exit 1
