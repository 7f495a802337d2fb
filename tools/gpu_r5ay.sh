#!/bin/bash
# Round 5: probe -- k_lib_raster without the split-tile (SHS_OPT_LIB_PART) path compiled
# (libshs_noparts.so; parts are off by default) against the default, C4 / C5 three times.
set -o pipefail
mkdir -p gpurun_out
VARIANTS="default noparts default noparts default noparts" CONFIGS="c4 c5" bash tools/exp_variants.sh || exit 1
