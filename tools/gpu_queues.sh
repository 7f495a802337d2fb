#!/bin/bash
# Frames in flight vs hardware queues: the 8-way region split of C4 / C5 (tools/exp_pipeline.py) with
# GPU_MAX_HW_QUEUES 4 (HIP's default) and 8, D = 3, 4, 6 frames in flight
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/queues.log
for q in 4 8; do for c in c5 c4; do
  echo "GPU_MAX_HW_QUEUES=$q" >> gpurun_out/queues.log
  GPU_MAX_HW_QUEUES=$q SPLIT_REGIONS=1 timeout -k 10 300 python -u tools/exp_pipeline.py $c 60 1,8 3,4,6 2>&1 | grep -v amdgpu.ids >> gpurun_out/queues.log || exit 1
done; done
cat gpurun_out/queues.log
