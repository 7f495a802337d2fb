#!/bin/bash
# Round 5: what the Forward+ light loop costs k_lib_resolve<5> (libshs_nolights.so: the loop skipped,
# wrong images) -- C4 bench A/B and the kernel trace of each.
set -o pipefail
mkdir -p gpurun_out
VARIANTS="default nolights default nolights" CONFIGS="c4" bash tools/exp_variants.sh || exit 1
for v in default nolights; do
  if [ $v = default ]; then L=; else L=$(pwd)/leisure-software-renderer_amd/shs_gpu/libshs_$v.so; fi
  SHS_GPU_LIB=$L bash tools/profile_kernels.sh r5ap_$v --config c4 > /dev/null 2>&1 || exit 1
  echo "== $v"; grep -A3 "isolated" gpurun_out/r5ap_${v}_kernel_timed.txt | grep -E "raster|resolve"
done
