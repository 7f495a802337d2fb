#!/bin/bash
# The switches below are read only by the timing-experiments build (make -C leisure-software-renderer_amd exp).
export SHS_GPU_LIB=${SHS_GPU_LIB:-$PWD/leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so}
# parity (library + legacy suites), then variant timing: C4 / C5 prev / heavy / default, C2 / C3 prev / default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_lib_parity.py tests/test_fullsize.py tests/test_regions.py tests/test_shipped_frames.py tests/test_light_parity.py tests/test_textures.py tests/test_shadow_footprint.py tests/test_shipped_regions.py tests/test_gather_gpu.py tests/test_gpu_parity.py tests/test_batch.py > gpurun_out/r4h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4h_tests.log; [ $rc -eq 0 ] || exit 1
VARIANTS="prev default prev default" CONFIGS="c5 c4" bash tools/exp_variants.sh || exit 1
# VARIANTS="prev default prev default" CONFIGS="c2 c3" bash tools/exp_variants.sh
# ENVS="SHS_GHOST_LIST=0 SHS_GHOST_LIST=1 SHS_GHOST_LIST=0 SHS_GHOST_LIST=1" CONFIG=c2 bash tools/exp_env.sh
