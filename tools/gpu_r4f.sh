#!/bin/bash
# deep camera raster with three barriers per pass: library parity suites, then C4 / C5 A/B against the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_lib_parity.py tests/test_fullsize.py tests/test_regions.py tests/test_shipped_frames.py tests/test_light_parity.py tests/test_textures.py tests/test_shadow_footprint.py tests/test_shipped_regions.py tests/test_gather_gpu.py > gpurun_out/r4f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4f_tests.log; [ $rc -eq 0 ] || exit 1
VARIANTS="prev default prev default" CONFIGS="c4 c5" bash tools/exp_variants.sh
