#!/bin/bash
# Library change A/B: library parity tests with the default build, then timing of the default build
# against shs_gpu/libshs_base.so (the previous commit) on CONFIGS (default c4 c5), interleaved twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_lib_parity.py \
  tests/test_fullsize.py tests/test_shipped_frames.py tests/test_light_parity.py tests/test_post.py tests/test_present.py \
  tests/test_regions.py tests/test_textures.py} > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
VARIANTS="base default base default" CONFIGS="${CONFIGS:-c4 c5}" bash tools/exp_variants.sh
