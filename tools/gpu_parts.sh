#!/bin/bash
# hot-tile parts (SHS_OPT_LIB_PART) with the round-4 raster: C4 at N = 1 and the 8-way region split
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/parts.log
for p in 0 256 512 1024; do
  echo "SPLIT_PART=$p" >> gpurun_out/parts.log
  SPLIT_PART=$p SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c4 60 1,8 3 2>&1 | grep "frames in flight" >> gpurun_out/parts.log || exit 1
done
cat gpurun_out/parts.log
