#!/bin/bash
# Round 5: C4 camera raster timelines (N = 1, rank 3 of 8 regions) and the resolve latency variants
# (libshs_pref / spec / both against the default build) on C4 / C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/timeline_lib.py c4 > gpurun_out/r5d_tl_c4_n1.log 2>&1 || exit 1
SPLIT_REGIONS=1 timeout -k 10 120 python -u tools/timeline_lib.py c4 1000 1000 8 3 > gpurun_out/r5d_tl_c4_r3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5d_tl_c4_n1.log gpurun_out/r5d_tl_c4_r3.log
VARIANTS="default pref spec both default pref spec both" CONFIGS="c4 c5" bash tools/exp_variants.sh
