#!/bin/bash
# Strong-scaling split on one GPU (round 4): every rank of the 8-way region-sharded C4 / C5 frame
# measured in turn with 3 frames in flight, N = 1 beside it, then rank 0 with the gather's 7 unpacks.
set -o pipefail
mkdir -p gpurun_out
for c in c5 c4; do
  SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 60 1,8 3 > gpurun_out/split_$c.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/exp_root.py $c 8 0.85 60 3 > gpurun_out/root_$c.log 2>&1 || exit 1
done
SPLIT_FOOTPRINT=0 SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py c5 60 1,8 3 > gpurun_out/split_c5_full.log 2>&1 || exit 1
cat gpurun_out/split_c5.log gpurun_out/root_c5.log gpurun_out/split_c5_full.log gpurun_out/split_c4.log gpurun_out/root_c4.log | grep -v amdgpu.ids
