#!/bin/bash
# Round 5: the Forward+ uniform light loop two lights per iteration (libshs_lp2.so, -DSHS_LIGHT_PAIRS)
# against the default: C4 parity with the variant, then C4 / C5 A/B three times.
set -o pipefail
mkdir -p gpurun_out
SHS_GPU_LIB=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_lp2.so timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_fullsize.py tests/test_lib_parity.py tests/test_light_parity.py > gpurun_out/r5au_tests.log 2>&1 || { tail -30 gpurun_out/r5au_tests.log; exit 1; }
grep -E "not bit-identical|passed|failed" gpurun_out/r5au_tests.log | tail -4
VARIANTS="default lp2 default lp2 default lp2" CONFIGS="c4" bash tools/exp_variants.sh || exit 1
