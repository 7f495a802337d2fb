#!/bin/bash
# Round 5: the split-tile path a compile-time k_lib_raster parameter (working tree) against HEAD
# (libshs_base.so): library parity (split parts included), C4 / C5 A/B three times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_lib_parity.py tests/test_fullsize.py tests/test_shipped_regions.py tests/test_shadow_footprint.py tests/test_textures.py > gpurun_out/r5az_tests.log 2>&1 || { tail -30 gpurun_out/r5az_tests.log; exit 1; }
tail -1 gpurun_out/r5az_tests.log
VARIANTS="base default base default base default" CONFIGS="c4 c5" bash tools/exp_variants.sh || exit 1
